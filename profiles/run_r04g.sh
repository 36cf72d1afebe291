#!/bin/bash
# Round-4 profiles on the generator-v2 build: extraction trace + FETCH/WRITE + SQ passes (bench.py reads the newest
# pmc_*/sq_* summaries), the K4 build's per-dispatch FETCH/WRITE (probes/k4_probe.py), and a kernel trace of the
# config-4 exact lane (bench_match.py). Every step has its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
bash profiles/run_rocprof.sh r04g > gpurun_out/r04g/prof.log 2>&1
bash profiles/run_sq.sh r04g > gpurun_out/r04g/sq.log 2>&1
OUT=gpurun_out/r04g/k4
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- python3 probes/k4_probe.py --reps 1 > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r04g/match -o run --output-format csv -- python3 bench_match.py --no-cpu --category-queries 200 > gpurun_out/r04g/match.json 2> gpurun_out/r04g/match.err
timeout -k 10 200 python3 probes/k2_stamps_probe.py > gpurun_out/r04g/k2_stamps.json 2> gpurun_out/r04g/k2_stamps.err
echo done
