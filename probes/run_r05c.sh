#!/bin/bash
# r05c: StreamBank / batched K6 tests, lane-parity tests, the bench line with the new stream leg, then the r04y
# service command once more under rocprofv3 (ordered teardown in place; last, it may dump core).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_resample.py tests/test_gpu_lane_parity.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -40 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/svc -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream --service-tracks 1000 --service-requests 256 > $O/svc.json 2> $O/svc.err
echo "svc rc=$?"
echo done
