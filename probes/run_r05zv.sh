#!/bin/bash
# r05zv: is the large-plane cost of K1/K2 address translation? The catalog shape (1024 x 30 s) extracted
# with the power plane bounded at 0.75 GB, at the engine's 3 GB default, and whole (one 10.8 GB group): timing first
# (the engine's kernel events), then one PMC pass per plane size with the TCP's UTCL1 request / hit / miss counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05zv
mkdir -p $O
for r in 1; do
  for rows in 196608 0 4194304; do
    timeout -k 10 120 python3 probes/k1_shape_probe.py --rounds 1 --seconds 1.5 --shapes 1024x30 --plane-rows $rows >> $O/timing.jsonl 2>> $O/timing.err || exit 4
  done
done
for rows in 196608 0 4194304; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum -d $O/pmc_$rows -o run --output-format csv -- python3 probes/k1_shape_probe.py --rounds 1 --seconds 0.3 --shapes 1024x30 --plane-rows $rows > $O/pmc_$rows.out 2> $O/pmc_$rows.err || exit 5
done
echo done
