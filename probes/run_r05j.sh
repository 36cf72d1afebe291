#!/bin/bash
# r05j: the full GPU suite, smoke and the bench line on the four-workgroup K5 build, then the K5 trace and
# FETCH/WRITE passes of the config-4 lane (bench.py catalog leg) for profiles/pmc_r05j_k5.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -40 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 4
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 5; }
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-service --no-stream"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- $B > $O/trace.json 2> $O/trace.err || exit 6
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/fetch -o run --output-format csv -- $B > $O/fetch.json 2> $O/fetch.err || exit 7
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/write -o run --output-format csv -- $B > $O/write.json 2> $O/write.err || exit 8
echo done
