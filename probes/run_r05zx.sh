#!/bin/bash
# r05zx: the exact lane (100k-track index, 10,000 clips, 4,096-clip aid_exact_lane calls) at the default 3 GiB
# K1 -> K2 plane bound against 2 GiB (524,288 rows) and 1.5 GiB, interleaved twice on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zx
mkdir -p $O
for i in 1 2; do
  for rows in 0 524288 393216; do
    timeout -k 10 240 python -u bench_match.py --no-cpu --category-queries 100 --plane-rows $rows > $O/lane_${rows}_$i.json 2>>$O/err.txt || exit 4
  done
done
echo done
