#!/bin/bash
# Level/band robustness GPU test, config 5 streaming (48 kHz and 16 kHz index), config 4 exact lane on the round-3 build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 bench_stream.py > $O/stream48.json 2> $O/stream48.err
timeout -k 10 300 python3 bench_stream.py --index-sr 16000 > $O/stream16.json 2> $O/stream16.err
timeout -k 10 400 python3 bench_match.py > $O/match.json 2> $O/match.err
echo done
