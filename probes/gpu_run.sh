#!/bin/bash
# One GPU-box run of the checked-in tree: probes/gpu_run.sh TAG STEP... with STEP one of
#   tests  the whole -m gpu suite        smoke  __graft_entry__.smoke()
#   bench  the default bench.py line     music  probes/music_eval.py (1,000 songs, 8 degradation categories)
#   prof   rocprofv3 --kernel-trace --stats of the headline-only bench
# Every step has its own time limit; the first failing step ends the run (exit 10 + step number).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?usage: gpu_run.sh TAG STEP...}
shift
O=gpurun_out/$TAG
mkdir -p $O
i=0
for step in "$@"; do
  i=$((i + 1))
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 ;;
    bench) timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err ;;
    music) timeout -k 10 900 python3 -u probes/music_eval.py --tracks 1000 --queries 500 --negatives 100 --workers 16 > $O/music.json 2> $O/music.err ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-catalog --no-stream --no-service > $O/prof_bench.json 2> $O/prof.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  [ $rc -eq 0 ] || exit $((10 + i))
done
echo done
