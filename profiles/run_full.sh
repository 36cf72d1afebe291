#!/bin/bash
# Round-end consolidated GPU run: full GPU test suite, smoke, headline bench, rocprofv3 trace and
# FETCH/WRITE passes (tag $1), config 4 and 5 benches. Every step has its own time limit.
set -e
TAG=${1:-r01k}
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err
bash profiles/run_rocprof.sh $TAG > gpurun_out/full_prof.log 2>&1
timeout -k 10 300 python bench_match.py > gpurun_out/full_match.json 2> gpurun_out/full_match.err
timeout -k 10 300 python bench_stream.py > gpurun_out/full_stream48.json 2> gpurun_out/full_stream48.err
timeout -k 10 300 python bench_stream.py --index-sr 16000 > gpurun_out/full_stream16.json 2> gpurun_out/full_stream16.err
timeout -k 10 300 python bench_catalog.py > gpurun_out/full_catalog.json 2> gpurun_out/full_catalog.err
