#!/bin/bash
# r05x: K6 integer decimation with 3 consecutive outputs per thread (one input walk; 4 per thread was 4-way bank-conflicted): resample / stream tests, then the
# stream leg under a kernel trace (r05w is the same command on the previous K6).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resample.py tests/test_gpu_stream.py -x -v --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-service > $O/bench.json 2> $O/bench.err || exit 5
echo done
