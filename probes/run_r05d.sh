#!/bin/bash
# r05d: K5 LDS path on 2-B posting signatures -- match/exact/lane-parity/stream GPU tests, an interleaved same-box
# A/B against the previous build (audio-ident_amd/build/prev_r05a) on the config-4 lane, then the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_exact.py tests/test_gpu_lane_parity.py tests/test_gpu_stream.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo tests failed; tail -40 $O/gpu_tests.txt; exit 3; }
tail -3 $O/gpu_tests.txt
bash probes/run_ab_k5.sh $O/k5_ab.txt prev_r05a 2 || exit 4
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -5 $O/bench.err; exit 5; }
echo done
