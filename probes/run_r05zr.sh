#!/bin/bash
# r05zr: config-4 lane call size above 4096 clips, alternated with 4096 on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zr
mkdir -p $O
for i in 1 2; do
  for b in 4096 8192; do
    timeout -k 10 300 python bench.py --no-cpu --no-fullband --no-service --no-stream --steps 3 --warmup 1 --exact-batch $b > $O/lane_${b}_$i.json 2>>$O/err.txt || exit 4
  done
done
echo done
