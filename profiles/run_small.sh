#!/bin/bash
# small-batch latency sizing (K1 min frames per wave, K2 min strip): parity tests, stream bench before/after,
# headline A/B. build/pre = the previous sizing.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/small
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_extract.py tests/test_gpu_exact.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/small/tests.log 2>&1 || { tail -20 gpurun_out/small/tests.log; exit 1; }
tail -1 gpurun_out/small/tests.log
timeout -k 10 300 python3 bench_stream.py > gpurun_out/small/stream_new.json 2>/dev/null || exit 1
AIDFP_LIB=$PWD/audio-ident_amd/build/pre/libaidfp.so timeout -k 10 300 python3 bench_stream.py > gpurun_out/small/stream_pre.json 2>/dev/null || exit 1
cat gpurun_out/small/stream_new.json gpurun_out/small/stream_pre.json
bash profiles/run_ab2.sh 2 main pre
