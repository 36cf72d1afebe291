#!/bin/bash
# K1 explicit vmcnt(0) before the power stores (the next frame's ring loads no longer wait behind this frame's hot
# stores): extraction parity tests on the new build, then a same-box A/B of HEAD (base), K2-only (k2) and the new build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  for v in base k2; do
    AIDFP_LIB=audio-ident_amd/build/$v/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_${v}_$r.json 2>/dev/null
  done
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
done
echo done
