#!/bin/bash
# r05w: kernel trace of the stream leg (256 live streams, 2.5 s pushes): where a push's time goes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-service > $O/bench.json 2> $O/bench.err || exit 4
echo done
