#!/bin/bash
# r05q: K4 with the column apply fused into the scatter (groups of 16 tiles) against the offs-matrix build
# (AID_K4_FUSED=0); CSR layout + sort-build tests on the product first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -k "csr_layout or sort_build" -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
for i in 1 2; do
for lib in product k4unfused; do
  if [ $lib = product ]; then unset AIDFP_LIB; else export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so; fi
  timeout -k 10 200 python3 probes/k4_probe.py --modes radix,radix_ballot,radix_again --reps 3 > $O/k4_${lib}_$i.json 2> $O/k4_${lib}_$i.err || exit 5
done
done
unset AIDFP_LIB
echo done
