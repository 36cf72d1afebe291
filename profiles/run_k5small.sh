cd "$GRAFT_REPO_ROOT"
for T in 10000 30000; do
for v in AIDFP_K5_LHIST=0 AIDFP_K5_LHIST=1 AIDFP_K5_LHIST=0 AIDFP_K5_LHIST=1; do
  env $v timeout -k 10 200 python3 bench_match.py --tracks $T > gpurun_out/k5s.json 2> gpurun_out/k5s.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/k5s.json').read().strip().splitlines()[-1]); print($T, '$v', d['value'], d['gpu_s'], d['top1_accuracy'], d['false_positive_rate'])"
done; done
