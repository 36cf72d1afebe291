#!/bin/bash
# K2 with one live pending candidate per thread (k2p1: 98 VGPRs instead of 120, 5 waves per SIMD): extraction parity
# tests on the variant, then a same-box A/B against the build on the bench and full-band data.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k
mkdir -p $O
V=audio-ident_amd/build/k2p1/libaidfp.so
AIDFP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests_k2p1.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_base_$r.json 2>/dev/null
  AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_k2p1_$r.json 2>/dev/null
done
echo done
