set -o pipefail
mkdir -p gpurun_out/r04f
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04f/gpu_tests.txt 2>&1; rc=$?
echo tests rc=$rc; tail -3 gpurun_out/r04f/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench_stream.py --index-sr 16000 --minutes 5 > gpurun_out/r04f/stream16_src441.json 2>gpurun_out/r04f/stream.err || exit 3
timeout -k 10 200 python bench_stream.py > gpurun_out/r04f/stream48.json 2>>gpurun_out/r04f/stream.err || exit 4
timeout -k 10 300 python bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04f/k4prof -o k4 -- python probes/k4_probe.py --reps 3 > gpurun_out/r04f/k4_probe.json 2> gpurun_out/r04f/k4_probe.err || exit 6
echo all ok
timeout -k 10 200 python probes/k2_stamps_probe.py > gpurun_out/r04f/k2_stamps.json 2> gpurun_out/r04f/k2_stamps.err || exit 7
echo stamps ok
