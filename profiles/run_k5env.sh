#!/bin/bash
# config 4 (bench_match.py) under environment settings. usage: bash profiles/run_k5env.sh "VAR=a" "VAR=b" ... ("-" = none)
cd "$GRAFT_REPO_ROOT"
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = "-" ]; then timeout -k 10 200 python3 bench_match.py > gpurun_out/k5env_$i.json 2> gpurun_out/k5env_$i.err || exit 1
  else env $v timeout -k 10 200 python3 bench_match.py > gpurun_out/k5env_$i.json 2> gpurun_out/k5env_$i.err || exit 1; fi
  python3 -c "import json; d=json.loads(open('gpurun_out/k5env_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['gpu_s'], d['top1_accuracy'], d['false_positive_rate'])"
done
