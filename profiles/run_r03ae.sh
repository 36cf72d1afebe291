#!/bin/bash
# rocprofv3 kernel trace + stats over the whole default bench line (extraction, full-band, catalog ingest with the
# K4 radix build, the config-4 exact lane), so every kernel the driver's line runs has a committed summary.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu > $O/bench.json 2> $O/bench.err
find $O -name '*stats*.csv'
echo done
