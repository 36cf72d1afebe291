set -o pipefail
mkdir -p gpurun_out/r04l
cd $GRAFT_REPO_ROOT
for v in product k5u8 k5u16 product; do
  if [ $v = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$v/libaidfp.so"; fi
  echo "== $v" >> gpurun_out/r04l/k5u_ab.txt
  env $L timeout -k 10 300 python3 probes/k5_path_probe.py --reps 4 >> gpurun_out/r04l/k5u_ab.txt 2>> gpurun_out/r04l/k5u_ab.err || exit 3
done
echo ok
