#!/bin/bash
# K2 hot words by vector load (no scalar load drained at the staging barrier) + range-checked buffer row loads:
# extraction parity tests on the new build, then a same-box A/B against the HEAD build (build/base).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
B=audio-ident_amd/build/base/libaidfp.so
for r in 1 2; do
  AIDFP_LIB=$B timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_base_$r.json 2>/dev/null
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
done
echo done
