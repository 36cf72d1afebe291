#!/bin/bash
# r05b: new GPU tests (lane parity, checksum, shard parity) + the existing match/comm/adapter tests, the FETCH_SIZE
# calibration probe for K5's 8-B reads, and one full default bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lane_parity.py tests/test_gpu_match.py tests/test_gpu_comm.py tests/test_gpu_adapter.py tests/test_gpu_concurrency.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -T -d $O/calib -o run --output-format csv -- probes/fetch_calib > $O/calib.out 2> $O/calib.err || exit 4
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 5; }
echo done
