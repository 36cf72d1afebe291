#!/bin/bash
# K1 real split on DPP partners (no E3 LDS exchange): the whole GPU suite, then a same-box A/B against the
# previous K1 (build/k1old) on the bench and full-band data, then the K1 kernel trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 120 --timeout-method thread > $O/tests_extract.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_new_$r.json 2>/dev/null
  AIDFP_LIB=audio-ident_amd/build/k1old/libaidfp.so timeout -k 10 120 python3 bench.py --no-cpu --no-catalog --steps 50 > $O/ab_old_$r.json 2>/dev/null
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-catalog --steps 20 > $O/prof_bench.json 2> $O/prof.err
echo done
