#!/bin/bash
# Round-3 consolidated run, part 2: config 4 (exact lane + robustness categories), config 5 (48 kHz index and a
# 16 kHz index through K6), config 3 (catalog bench), the K4 probe under the tracer, the concurrency probe.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 500 python bench_match.py > $O/match.json 2> $O/match.err
timeout -k 10 300 python bench_stream.py > $O/stream48.json 2> $O/stream48.err
timeout -k 10 300 python bench_stream.py --index-sr 16000 > $O/stream16.json 2> $O/stream16.err
timeout -k 10 300 python bench_catalog.py > $O/catalog.json 2> $O/catalog.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4 -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4.json 2> $O/k4.err
timeout -k 10 300 python3 probes/concurrency_probe.py > $O/concurrency.json 2> $O/concurrency.err
echo done
