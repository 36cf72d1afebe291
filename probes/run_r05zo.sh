#!/bin/bash
# r05zo: extraction kernel time per audio-second for catalog batch sizes (30 s tracks), shapes interleaved.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zo
mkdir -p $O
timeout -k 10 200 python -u probes/k1_shape_probe.py --rounds 2 --seconds 1 --shapes 128x30,256x30,512x30,1024x30 > $O/shape.jsonl 2>$O/err.txt || exit 4
for b in 256 512 1024; do
  timeout -k 10 150 python -u probes/catalog_async_ab.py --sr 44100 --reps 2 --batch $b >> $O/catalog.jsonl 2>>$O/err.txt || exit 5
done
echo done
