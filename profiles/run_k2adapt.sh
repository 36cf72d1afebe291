#!/bin/bash
# K2 adaptive strip sizing: extraction/exact/match parity, then band-limited vs full-band timing for the
# adaptive sizing and fixed multipliers, then the bench A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_extract.py tests/test_gpu_exact.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/k2a_tests.log 2>&1 || { tail -20 gpurun_out/k2a_tests.log; exit 1; }
tail -1 gpurun_out/k2a_tests.log
for x in "" 1 1.5; do
  if [ -z "$x" ]; then timeout -k 10 120 python3 probes/fullband_probe.py || exit 1
  else AIDFP_K2_SLOTS_X=$x timeout -k 10 120 python3 probes/fullband_probe.py || exit 1; fi
done
bash profiles/run_ab_env.sh 3 "-" "AIDFP_K2_SLOTS_X=1"
