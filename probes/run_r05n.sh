#!/bin/bash
# r05n: LDS same-address atomic lane order (probes/lds_atomic_order.hip), the CSR layout test on the product build,
# and the same test on the timing-only one-atomic-rank K4 build (AID_K4_DIAG=4: is it a stable rank in practice?).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 120 probes/lds_atomic_order 4096 256 > $O/order.json 2> $O/order.err || exit 4
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -k csr_layout -x -v --timeout 200 --timeout-method thread > $O/csr_product.txt 2>&1 || exit 5
export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/k4diag4/libaidfp.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -k "csr_layout and sort" -v --timeout 200 --timeout-method thread > $O/csr_diag4.txt 2>&1
echo "diag4 rc $?" >> $O/csr_diag4.txt
echo done
