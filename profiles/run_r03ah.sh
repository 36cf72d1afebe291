#!/bin/bash
# K2 candidate test as two compares (p > before, p >= right: SGPR masks + s_and) instead of add + max + one compare.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash profiles/run_variants.sh 5 main k2c2 > gpurun_out/r03ah_ab.txt 2>&1
echo done
