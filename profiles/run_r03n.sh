#!/bin/bash
# K1 two frames per wave (AID_K1_PAIR build): extraction parity tests on the variant, then a same-box A/B against the
# current build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03n
mkdir -p $O
V=audio-ident_amd/build/k1pair/libaidfp.so
AIDFP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
  AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_pair_$r.json 2>/dev/null
done
echo done
