set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err
bash profiles/run_rocprof.sh r01k > gpurun_out/full_prof.log 2>&1
