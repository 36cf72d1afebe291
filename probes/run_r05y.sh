#!/bin/bash
# r05y: the extraction profiles of the round-5 build (the r05z passes also caught the new stream leg's launches):
# kernel trace + FETCH / WRITE passes and the SQ passes of the headline bench only.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash profiles/run_rocprof.sh r05y > gpurun_out/r05y_prof.log 2>&1
bash profiles/run_sq.sh r05y > gpurun_out/r05y_sq.log 2>&1
echo done
