#!/bin/bash
# Profiles of the round's final build (tag r03zf sorts after r03y, so bench.py reads these): rocprofv3 kernel
# trace + stats, FETCH_SIZE and WRITE_SIZE passes, SQ issue/occupancy passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03zf
bash profiles/run_rocprof.sh r03zf > gpurun_out/r03zf/prof.log 2>&1
bash profiles/run_sq.sh r03zf > gpurun_out/r03zf/sq.log 2>&1
echo done
