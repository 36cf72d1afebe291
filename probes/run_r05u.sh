#!/bin/bash
# r05u: K2 with the packed vertical state (AID_K2_PACKPEND: 112 VGPRs at 4 workgroups per CU, 96 + 9 spilled at 5)
# against the product: K2 extraction tests on each variant, then the band-limited / full-band timing, 3 rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05u
mkdir -p $O
for lib in k2pp4 k2pp5; do
  export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests_$lib.txt 2>&1 || exit 4
done
for i in 1 2 3; do
for lib in product k2pp4 k2pp5; do
  if [ $lib = product ]; then unset AIDFP_LIB; else export AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so; fi
  echo "== $lib $i" >> $O/k2.txt
  timeout -k 10 200 python3 probes/fullband_probe.py 0 >> $O/k2.txt 2>> $O/k2.err || exit 5
done
done
unset AIDFP_LIB
echo done
