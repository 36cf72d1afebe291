#!/bin/bash
# r05zi: catalog ingest at bench.py's 44.1 kHz: A/B of the asynchronous append (baseline library vs this tree) and
# the per-kernel breakdown of one pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zi
mkdir -p $O
for i in 1 2; do
  AIDFP_LIB=probes/ab/libaidfp_r05base.so timeout -k 10 200 python -u probes/catalog_async_ab.py --sr 44100 --wait-synth >> $O/ab.jsonl 2>>$O/ab.err || exit 5
  timeout -k 10 200 python -u probes/catalog_async_ab.py --sr 44100 >> $O/ab.jsonl 2>>$O/ab.err || exit 6
done
timeout -k 10 200 python -u probes/catalog_async_ab.py --sr 44100 --reps 1 --profile >> $O/ab.jsonl 2>>$O/ab.err || exit 7
echo done
