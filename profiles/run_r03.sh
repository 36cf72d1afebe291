#!/bin/bash
# Round-3 GPU run (tag $1): GPU tests, smoke, the headline bench (N=1, with the full-band and config-3 keys),
# a 2-rank rehearsal of the N>1 path on one GPU (gloo), and the rocprofv3 kernel trace. Each step has its
# own time limit; the first failure ends the call (set -e).
set -e
TAG=${1:-r03a}
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
AIDFP_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu --catalog-tracks 20000 > $O/bench_gloo2.json 2> $O/bench_gloo2.err
bash profiles/run_rocprof.sh $TAG > $O/prof.log 2>&1
echo done
