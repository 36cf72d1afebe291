#!/bin/bash
# K4: run ends written by the last scatter pass (no key array, no run-end kernel), plus two store experiments on the
# first passes (k4nt: non-temporal stores; k4swapv: pass 1 writes the other value buffer); build/k4xcd = the previous
# commit. Match parity tests for each build, then the K4 probe under the tracer for each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
B=audio-ident_amd/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_comm.py tests/test_gpu_exact.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
AIDFP_LIB=$B/k4nt/libaidfp.so timeout -k 10 200 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > $O/tests_k4nt.log 2>&1
AIDFP_LIB=$B/k4swapv/libaidfp.so timeout -k 10 200 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > $O/tests_k4swapv.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4new -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4new.json 2> $O/k4new.err
for v in k4nt k4swapv k4xcd; do
  AIDFP_LIB=$B/$v/libaidfp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 probes/k4_probe.py > $O/$v.json 2> $O/$v.err
done
echo done
