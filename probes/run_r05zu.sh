#!/bin/bash
# r05zu: the tree as rebuilt in a re-created container (same sources as r05zt): whole GPU suite, smoke, the default
# bench line, then a kernel-trace summary of the headline leg alone.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zu
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 4
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 5
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu --no-fullband --no-catalog --no-stream --no-service > $O/bench_prof.json 2> $O/bench_prof.err || exit 7
echo done
