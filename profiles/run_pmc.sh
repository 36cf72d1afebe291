#!/bin/bash
# One rocprofv3 PMC pass over a short bench run. usage: bash profiles/run_pmc.sh <outdir> <counters...>
set -e
OUTD=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$OUTD
timeout -k 10 300 rocprofv3 --pmc "$@" -T -d gpurun_out/$OUTD -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-service --no-stream > gpurun_out/$OUTD/log 2>&1
