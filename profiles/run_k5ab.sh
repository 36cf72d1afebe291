cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-main k5d1 k5d2}; do
  L=$PWD/audio-ident_amd/aidfp/libaidfp.so; [ $v != main ] && L=$PWD/audio-ident_amd/build/$v/libaidfp.so
  AIDFP_LIB=$L timeout -k 10 200 python3 bench_match.py > gpurun_out/k5ab_$v.json 2> gpurun_out/k5ab_$v.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/k5ab_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['gpu_s'])"
done
