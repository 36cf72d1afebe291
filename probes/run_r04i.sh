set -o pipefail
mkdir -p gpurun_out/r04i
cd $GRAFT_REPO_ROOT
for v in product k4s8 k4c1024 product; do
  if [ $v = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$v/libaidfp.so"; fi
  env $L timeout -k 10 200 python3 probes/k4_probe.py --reps 4 --modes radix >> gpurun_out/r04i/k4_ab.jsonl 2>> gpurun_out/r04i/k4_ab.err || exit 3
done
echo ok
