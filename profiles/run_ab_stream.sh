#!/bin/bash
# Interleaved A/B of bench_stream.py (K5 LDS path against a 1000-track index) per library variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abs
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@"; do
    LIBP=audio-ident_amd/aidfp/libaidfp.so; [ "$v" != main ] && LIBP=audio-ident_amd/build/$v/libaidfp.so
    AIDFP_LIB=$PWD/$LIBP timeout -k 10 200 python3 bench_stream.py > gpurun_out/abs/${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(tail -1 gpurun_out/abs/${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["push_latency_ms"])')"
  done
done
