#!/bin/bash
# K4 radix v3: match parity tests (every K4 build) + the K4 A/B probe under the tracer; concurrent readers
# (64 in flight == serial) + their latency probe; then a same-box A/B on the bench and full-band data of
# base (K1 twiddle pairs as b128), k1old (the previous commit) and k2d2 (K2 prefetch depth 2).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_comm.py tests/test_gpu_concurrency.py tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/k4 -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4.json 2> $O/k4.err
timeout -k 10 240 python3 probes/concurrency_probe.py > $O/concurrency.json 2> $O/concurrency.err
V=audio-ident_amd/build/k2d2/libaidfp.so
AIDFP_LIB=$V timeout -k 10 200 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 200 --timeout-method thread > $O/tests_k2d2.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_base_$r.json 2>/dev/null
  AIDFP_LIB=audio-ident_amd/build/k1old/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_k1old_$r.json 2>/dev/null
  AIDFP_LIB=$V timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_k2d2_$r.json 2>/dev/null
done
echo done
