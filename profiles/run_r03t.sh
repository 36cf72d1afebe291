#!/bin/bash
# K2 with the next row's LDS window data read one row ahead (occupancy 4 with a small spill, or 3), parity tests on
# each, then an ABBA bench A/B against the current build (2e8ff62's K2 = build/prev).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t
mkdir -p $O
for v in k2la4 k2la3; do
  AIDFP_LIB=audio-ident_amd/build/$v/libaidfp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1
done
for v in prev k2la4 k2la3 k2la3 k2la4 prev; do
  n=$(ls $O | grep -c "ab_${v}_" || true)
  AIDFP_LIB=audio-ident_amd/build/$v/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$((n+1)).json 2>/dev/null
done
echo done
