#!/bin/bash
# K2 -> K3 per-frame peak counts (K3 phase 1 reads one u32 per frame instead of 16 mask words): extraction parity
# tests, then a same-box A/B against 2e8ff62 (build/prev).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py tests/test_gpu_exact.py tests/test_gpu_adapter.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  AIDFP_LIB=audio-ident_amd/build/prev/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_prev_$r.json 2>/dev/null
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
done
echo done
