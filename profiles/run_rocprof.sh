#!/bin/bash
# rocprofv3 passes for one round: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes.
# usage: bash tools_prof.sh <tag>
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle 0 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --settle 0 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $OUT/write.log 2>&1
find $OUT -name '*.csv' | head -20
