#!/bin/bash
# K2 mask words stored by lane 0 as two 16-B stores (data by 4 v_mov_b64 of the SGPR ballots) instead of 8 v_writelane + a 4-lane store.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash profiles/run_variants.sh 5 main k2l0 > gpurun_out/r03am_ab.txt 2>&1
echo done
