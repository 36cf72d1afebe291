#!/bin/bash
# 2-rank gloo rehearsal of the N>1 bench line (two ranks share the one GPU), now with the exact-lane leg.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ad
mkdir -p $O
AIDFP_BENCH_BACKEND=gloo timeout -k 10 700 python -u bench.py --gpus 2 --no-cpu > $O/bench.json 2> $O/bench.err
echo done
