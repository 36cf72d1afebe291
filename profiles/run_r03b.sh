#!/bin/bash
# 16-bin hot chunks (K1 -> K2): extraction parity tests + bench; K4 build A/B (hand radix vs rocPRIM vs atomic)
# under the kernel tracer; bench_match (config 4 with the match roofline and the robustness categories) and its
# kernel trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-catalog > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/k4 -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4.json 2> $O/k4.err
timeout -k 10 400 python3 bench_match.py > $O/match.json 2> $O/match.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/match_prof -o run --output-format csv -- python3 bench_match.py --queries 4096 --category-queries 0 > $O/match_prof.json 2> $O/match_prof.err
echo done
