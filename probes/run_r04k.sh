set -o pipefail
mkdir -p gpurun_out/r04k
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_exact.py tests/test_gpu_concurrency.py tests/test_gpu_stream.py tests/test_gpu_adapter.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04k/gpu_tests.txt 2>&1; rc=$?
echo tests rc=$rc; tail -2 gpurun_out/r04k/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 probes/k5_path_probe.py > gpurun_out/r04k/k5_path.json 2> gpurun_out/r04k/k5_path.err || exit 4
timeout -k 10 300 python bench.py > gpurun_out/r04k/bench.json 2> gpurun_out/r04k/bench.err || exit 5
echo all ok
