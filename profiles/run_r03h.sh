#!/bin/bash
# CSR bucket key as an entropy-balanced bit permutation (aidfp_layout.h bucket_key): the whole GPU suite, the K4
# probe for this build and the previous one (build/k4xcd) under the tracer, and config 4 (match rows and accuracy).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4new -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4new.json 2> $O/k4new.err
AIDFP_LIB=audio-ident_amd/build/k4xcd/libaidfp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k4old -o run --output-format csv -- python3 probes/k4_probe.py > $O/k4old.json 2> $O/k4old.err
timeout -k 10 500 python3 bench_match.py --category-queries 0 > $O/match.json 2> $O/match.err
echo done
