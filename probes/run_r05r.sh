#!/bin/bash
# r05r: K4 count kernel with 16-B key loads against 4-B loads (AID_K4_CNTVEC=0); in each, the one-atomic rank against
# the ballot rank (k4_build 4); CSR layout + sort-build tests on the product first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -k "csr_layout or sort_build" -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
for i in 1 2 3; do
for lib in product k4cnt4; do
  if [ $lib = product ]; then unset AIDFP_LIB; else export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so; fi
  timeout -k 10 200 python3 probes/k4_probe.py --modes radix,radix_ballot,radix_again --reps 3 > $O/k4_${lib}_$i.json 2> $O/k4_${lib}_$i.err || exit 5
done
done
unset AIDFP_LIB
echo done
