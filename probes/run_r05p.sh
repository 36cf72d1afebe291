#!/bin/bash
# r05p: K4 scatter with its counters in the key staging area (52 KB, three workgroups per CU) against the 61 KB
# two-per-CU build (AID_K4_LDS3=0), both with the one-atomic rank; CSR layout + sort-build tests on the product first.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -k "csr_layout or sort_build" -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
for i in 1 2; do
for lib in product k4lds2; do
  if [ $lib = product ]; then unset AIDFP_LIB; else export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so; fi
  timeout -k 10 200 python3 probes/k4_probe.py --modes radix,radix_ballot,radix_again --reps 3 > $O/k4_${lib}_$i.json 2> $O/k4_${lib}_$i.err || exit 5
done
done
unset AIDFP_LIB
echo done
