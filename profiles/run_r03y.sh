#!/bin/bash
# Round-3 consolidated run on the current build: full GPU suite, smoke, headline bench (all legs), a same-box A/B
# against 2e8ff62 (build/prev: before the SCC clobber), rocprofv3 trace + FETCH/WRITE passes, SQ passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
for r in 1 2; do
  AIDFP_LIB=audio-ident_amd/build/prev/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_prev_$r.json 2>/dev/null
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
done
bash profiles/run_rocprof.sh r03y > $O/prof.log 2>&1
bash profiles/run_sq.sh r03y > $O/sq.log 2>&1
echo done
