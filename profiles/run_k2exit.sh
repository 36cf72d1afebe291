#!/bin/bash
# K2 strip-cold early exit (AID_K2_WCOLD_EXIT) with more strips per workgroup slot (AIDFP_K2_SLOTS_X).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
W=$PWD/audio-ident_amd/build/wexit/libaidfp.so
AIDFP_LIB=$W timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/k2exit_smoke.log 2>&1 || { echo "smoke FAILED"; tail -5 gpurun_out/k2exit_smoke.log; exit 1; }
AIDFP_LIB=$W AIDFP_K2_SLOTS_X=2 timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/k2exit_smoke.log 2>&1 || { echo "smoke x2 FAILED"; exit 1; }
AIDFP_LIB=$W AIDFP_K2_SLOTS_X=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_extract.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k2exit_tests.log 2>&1 || { tail -20 gpurun_out/k2exit_tests.log; exit 1; }
tail -1 gpurun_out/k2exit_tests.log
bash profiles/run_ab_env.sh 2 "-" "AIDFP_LIB=$W" "AIDFP_LIB=$W AIDFP_K2_SLOTS_X=1.5" "AIDFP_LIB=$W AIDFP_K2_SLOTS_X=2" "AIDFP_LIB=$W AIDFP_K2_SLOTS_X=3"
