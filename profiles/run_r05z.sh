#!/bin/bash
# Round-end consolidated run on the current build: GPU tests, smoke, bench (default line), profiles (trace, FETCH /
# WRITE, SQ) tagged $TAG, the K5 trace + FETCH/WRITE of the config-4 lane, config 4/5 benches, and the world-8 gloo
# rehearsal of the N-rank line. Each step has its own time limit; the first failure ends the script.
set -e
TAG=${1:-r05z}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
bash profiles/run_rocprof.sh $TAG > $O/prof.log 2>&1
bash profiles/run_sq.sh $TAG > $O/sq.log 2>&1
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-service --no-stream"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/k5/trace -o run --output-format csv -- $B > $O/k5_trace.json 2> $O/k5_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/k5/fetch -o run --output-format csv -- $B > $O/k5_fetch.json 2> $O/k5_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/k5/write -o run --output-format csv -- $B > $O/k5_write.json 2> $O/k5_write.err
timeout -k 10 300 python bench_match.py > $O/config4_match.json 2> $O/config4_match.err
timeout -k 10 200 python bench_stream.py --index-sr 16000 > $O/config5_stream16.json 2> $O/stream.err
AIDFP_BENCH_BACKEND=gloo timeout -k 10 700 python bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu --catalog-tracks 8000 --exact-clips 1000 --service-tracks 2000 --service-requests 128 --stream-count 32 --stream-tracks 2000 --stream-seconds 30 > $O/bench_gloo8_rehearsal.json 2> $O/bench_gloo8.err
echo done
