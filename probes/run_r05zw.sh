#!/bin/bash
# r05zw: the K1 -> K2 plane bound swept finer around the 3 GB default (786,432 rows of 4 KB), catalog shape
# 1024 x 30 s, two interleaved rounds, engine kernel events.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zw
mkdir -p $O
for r in 1 2; do
  for rows in 393216 589824 786432 1048576 1310720 1572864 2097152; do
    timeout -k 10 120 python3 probes/k1_shape_probe.py --rounds 1 --seconds 1.5 --shapes 1024x30 --plane-rows $rows >> $O/timing.jsonl 2>> $O/timing.err || exit 4
  done
done
echo done
