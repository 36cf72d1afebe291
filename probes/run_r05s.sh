#!/bin/bash
# r05s: exact-lane accuracy on host-generated music-like songs (probes/music_eval.py), independent of aidfp.synth.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 900 python3 -u probes/music_eval.py --tracks 1000 --queries 500 --negatives 100 --workers 16 > $O/music.json 2> $O/music.err || exit 4
echo done
