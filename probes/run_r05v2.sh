#!/bin/bash
# r05v2: run-to-run spread of the headline on one box: the default bench line once, then the extraction-only line 4x.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v2
mkdir -p $O
timeout -k 10 400 python bench.py > $O/full.json 2> $O/full.err || exit 4
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu --no-fullband --no-catalog --no-service --no-stream > $O/head_$i.json 2> $O/head_$i.err || exit 5
done
echo done
