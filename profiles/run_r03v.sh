#!/bin/bash
# Host-oracle baselines for configs 3 (bench.py cpu_baseline.catalog) and 4 (bench_match.py cpu_baseline), with the
# headline bench and the config-4 exact lane on the round-3 build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 600 python3 bench_match.py > $O/match.json 2> $O/match.err
echo done
