set -o pipefail
mkdir -p gpurun_out/r04h
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_comm.py tests/test_gpu_exact.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04h/gpu_tests.txt 2>&1; rc=$?
echo tests rc=$rc; tail -2 gpurun_out/r04h/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r04h/k4prof -o k4 --output-format csv -- python3 probes/k4_probe.py --reps 3 > gpurun_out/r04h/k4_probe.json 2> gpurun_out/r04h/k4_probe.err || exit 6
timeout -k 10 300 python bench.py > gpurun_out/r04h/bench.json 2> gpurun_out/r04h/bench.err || exit 5
echo all ok
