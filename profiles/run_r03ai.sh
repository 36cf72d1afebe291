#!/bin/bash
# K2 bin-0 exclusion as a uniform lane mask in the candidate test (SALU) instead of a per-lane max (VALU).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash profiles/run_variants.sh 5 main k2b0 > gpurun_out/r03ai_ab.txt 2>&1
echo done
