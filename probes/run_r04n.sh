set -o pipefail
mkdir -p gpurun_out/r04n
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_comm.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04n/gpu_tests.txt 2>&1; rc=$?
echo tests rc=$rc; tail -2 gpurun_out/r04n/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r04n/k4prof -o k4 --output-format csv -- python3 probes/k4_probe.py --reps 4 --modes radix,rocprim > gpurun_out/r04n/k4_probe.json 2> gpurun_out/r04n/k4_probe.err || exit 6
echo all ok
