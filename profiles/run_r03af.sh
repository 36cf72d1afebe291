#!/bin/bash
# K2 instruction trims A/B: v1 = no zero-init of the ballot-word registers (only lanes 0..3 are stored),
# v2 = v1 + the `before` maximum computed ahead of the ring update (the m7 phi copies coalesce away).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 bash profiles/run_variants.sh 4 main k2v1 k2v2 main > gpurun_out/r03af_ab.txt 2>&1
echo done
