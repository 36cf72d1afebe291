#!/bin/bash
# K4 radix with XCD-contiguous tiles: match parity tests, then the K4 probe (radix vs rocPRIM) for this build and the
# previous one (build/k1old) on the same box, under the kernel tracer.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4new -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4new.json 2> $O/k4new.err
AIDFP_LIB=audio-ident_amd/build/k1old/libaidfp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4old -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4old.json 2> $O/k4old.err
timeout -k 10 300 python3 probes/concurrency_probe.py > $O/concurrency.json 2> $O/concurrency.err
echo done
