#!/bin/bash
# Round-end consolidated run on the current build: GPU tests, smoke, bench (default line), profiles (trace, FETCH /
# WRITE, SQ) tagged r04zm, config 4/5 benches, and the world-8 gloo rehearsal of the N-rank line. Each step has its
# own time limit; the first failure ends the script.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04zm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
bash profiles/run_rocprof.sh r04zm > $O/prof.log 2>&1
bash profiles/run_sq.sh r04zm > $O/sq.log 2>&1
timeout -k 10 300 python bench_match.py > $O/config4_match.json 2> $O/config4_match.err
timeout -k 10 200 python bench_stream.py > $O/config5_stream48.json 2> $O/stream.err
timeout -k 10 200 python bench_stream.py --index-sr 16000 > $O/config5_stream16.json 2>> $O/stream.err
AIDFP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu --catalog-tracks 8000 --exact-clips 1000 --service-tracks 2000 --service-requests 128 > $O/bench_gloo8_rehearsal.json 2> $O/bench_gloo8.err
echo done
