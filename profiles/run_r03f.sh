#!/bin/bash
# Config 4 (exact lane vs the 100k catalog) with the match roofline and the robustness categories, its kernel
# trace, then K4's HBM bytes per dispatch (FETCH_SIZE and WRITE_SIZE in separate PMC passes over the A/B probe).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 500 python3 bench_match.py > $O/match.json 2> $O/match.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/match_prof -o run --output-format csv -- python3 bench_match.py --queries 4096 --category-queries 0 > $O/match_prof.json 2> $O/match_prof.err
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/k4fetch -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $O/k4fetch.json 2> $O/k4fetch.err
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/k4write -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $O/k4write.json 2> $O/k4write.err
echo done
