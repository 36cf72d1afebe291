#!/bin/bash
# Configs 4 and 5 on the round's final build: exact lane with its robustness categories and host baseline, and the
# 48 kHz stereo stream against a 48 kHz and a 16 kHz index.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03an
mkdir -p $O
timeout -k 10 600 python3 bench_match.py > $O/match.json 2> $O/match.err
timeout -k 10 300 python3 bench_stream.py > $O/stream48.json 2> $O/stream48.err
timeout -k 10 300 python3 bench_stream.py --index-sr 16000 > $O/stream16.json 2> $O/stream16.err
echo done
