#!/bin/bash
# r05zz2: is the K1 plane-bound knee a back-to-back effect? Catalog shape at 3 GiB and the whole plane, calls back to
# back against calls separated by a sync and a 20 ms idle gap, interleaved twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zz2
mkdir -p $O
for r in 1 2; do
  for rows in 786432 4194304; do
    for gap in 0 20; do
      timeout -k 10 120 python3 probes/k1_shape_probe.py --rounds 1 --seconds 1.5 --shapes 1024x30 --plane-rows $rows --gap-ms $gap >> $O/timing.jsonl 2>> $O/timing.err || exit 4
    done
  done
done
echo done
