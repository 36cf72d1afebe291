#!/bin/bash
# Round-3 consolidated run, part 1: full GPU suite, smoke, headline bench (all legs), rocprofv3 trace + FETCH/WRITE
# passes (tag r03x), SQ passes. Every GPU step has its own time limit; the steps are chained by set -e.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
bash profiles/run_rocprof.sh r03x > $O/prof.log 2>&1
bash profiles/run_sq.sh r03x > $O/sq.log 2>&1
echo done
