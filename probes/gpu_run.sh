#!/bin/bash
# One GPU-box run of the checked-in tree: probes/gpu_run.sh TAG STEP... with STEP one of
#   tests  the whole -m gpu suite        smoke  __graft_entry__.smoke()
#   bench  the default bench.py line     music  probes/music_eval.py (1,000 songs, 8 degradation categories)
#   prof   rocprofv3 --kernel-trace --stats of the headline-only bench
#   pmc    the headline's kernel trace, FETCH_SIZE / WRITE_SIZE and SQ passes (profiles/run_rocprof.sh, run_sq.sh:
#          gpurun_out/prof_TAG, gpurun_out/sq_TAG, the inputs of tools/prof_summary.py TAG)
#   k5     the config-4 lane (catalog leg): kernel trace, FETCH_SIZE, WRITE_SIZE (tools/k5_pmc_summary.py inputs)
#   k5req  the lane's memory-side read requests by size (TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B) and TCP->TCC reads
#   segv   VERDICT r5 #2: the r05y2 command (service leg under --kernel-trace --memory-copy-trace), once
#   counters  rocprofv3 -L
#   k2ab   interleaved same-box A/B of the product library vs audio-ident_amd/build/$K2AB_VARIANT (probes/run_ab_lib.sh, 3 rounds)
#   ctests the GPU tests of the service, its coalescer and the stream bank only
#   k6ab   the pipelined stream probe on the product library and the K6 variants in $K6AB_VARIANTS (build/<v>), 3 rounds
#   k2mall K1/K2 per step with the clip groups' power plane forced to fit the Infinity Cache (probes/k2_mall_probe.py)
#   gloo4  world-4 rehearsal of bench.py's N-rank path on the one GPU (gloo; RCCL refuses two ranks per GPU)
#   k6pmc  SQ, FETCH_SIZE and WRITE_SIZE passes over the 256-stream push probe (K6 and the windowed extraction)
#   k6res  bench_resample.py (256 x 10 s stereo 48 kHz -> 16 / 44.1 kHz) on the product and $K6AB_VARIANTS, 2 rounds
#   settleab headline only: (steps, settle seconds) = (20, 0.1), (100, 0.1), (100, 0.5), 3 interleaved rounds
#   k5ab   bench_match.py (config 4 lane) on the product and $K5AB_VARIANTS, 2 rounds
#   copyab the service leg with the PCM copy threaded from 16 MiB (product) or 8 MiB batches, 3 rounds
#   copythr the service leg with 4 or 8 PCM copy threads, 3 rounds
#   winab  the service leg with a 0.5 / 0.2 / 1.0 ms coalescing window, 3 rounds
#   splitab the service leg with split_min 16 / 8 / 32 (or $SPLITAB_MIN), 3 rounds
#   svc    the service leg alone (defaults)
#   mtests the match GPU tests only (K4/K5 parity, lane)
#   xtests the extraction GPU tests only (K1-K3 parity)
#   svcab  the service leg: synchronous dispatch, pipelined without / with batch splitting (16, 32), 2 rounds
#   streamprof  probes/stream_host_profile.py (256 streams: push wall time, GPU kernels per push, cProfile)
#   streamtrace the same probe under rocprofv3 --runtime-trace --kernel-trace (HIP API durations: host waits)
#   k5mm   config 4 (bench_match.py, 100k tracks, 10k + 1k clips) at engine min_match 10 and 12: K5 time, fallbacks
# Every step has its own time limit; the first failing step ends the run (exit 10 + step number).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?usage: gpu_run.sh TAG STEP...}
shift
O=gpurun_out/$TAG
mkdir -p $O
i=0
for step in "$@"; do
  i=$((i + 1))
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 ;;
    ctests) timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py tests/test_gpu_adapter.py tests/test_gpu_stream.py tests/test_gpu_resample.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_ctests.txt 2>&1 ;;
    mtests) timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_load.py tests/test_gpu_lane_parity.py tests/test_gpu_exact.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_mtests.txt 2>&1 ;;
    xtests) timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_xtests.txt 2>&1 ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 ;;
    bench) timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err ;;
    music) timeout -k 10 900 python3 -u probes/music_eval.py --tracks 1000 --queries 500 --negatives 100 --workers 16 > $O/music.json 2> $O/music.err ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-catalog --no-stream --no-service > $O/prof_bench.json 2> $O/prof.err ;;
    pmc) bash profiles/run_rocprof.sh $TAG > $O/pmc_prof.log 2>&1 && bash profiles/run_sq.sh $TAG > $O/pmc_sq.log 2>&1 ;;
    k5)
      B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-service --no-stream"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/k5/trace -o run --output-format csv -- $B > $O/k5_trace.json 2> $O/k5_trace.err &&
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/k5/fetch -o run --output-format csv -- $B > $O/k5_fetch.json 2> $O/k5_fetch.err &&
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/k5/write -o run --output-format csv -- $B > $O/k5_write.json 2> $O/k5_write.err ;;
    k5req)
      B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-service --no-stream"
      timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_READ_REQ_sum -T -d $O/k5/req -o run --output-format csv -- $B > $O/k5_req.json 2> $O/k5_req.err ;;
    segv) timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream > $O/segv.json 2> $O/segv.err ;;
    counters) timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 ;;
    k2ab) timeout -k 10 900 bash probes/run_ab_lib.sh $O/k2_ab.txt ${K2AB_VARIANT:?set K2AB_VARIANT} 3 > $O/k2ab.log 2>&1 ;;
    streamprof) timeout -k 10 300 python3 probes/stream_host_profile.py > $O/stream_prof.txt 2> $O/stream_prof.err ;;
    streamprofp) timeout -k 10 300 python3 probes/stream_host_profile.py --pipelined > $O/stream_prof_p.txt 2> $O/stream_prof_p.err ;;
    streamtracep) timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --stats -T -d $O/straceP -o run --output-format csv -- python3 probes/stream_host_profile.py --seconds 30 --pipelined > $O/stream_trace_p.txt 2> $O/stream_trace_p.err ;;
    streamtrace) timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --stats -T -d $O/strace -o run --output-format csv -- python3 probes/stream_host_profile.py --seconds 30 > $O/stream_trace.txt 2> $O/stream_trace.err ;;
    k5mm)
      timeout -k 10 400 python3 bench_match.py --no-cpu --category-queries 200 --min-match 10 > $O/k5mm10.json 2> $O/k5mm10.err &&
      timeout -k 10 400 python3 bench_match.py --no-cpu --category-queries 200 --min-match 12 > $O/k5mm12.json 2> $O/k5mm12.err ;;
    svcab)
      rc=0
      for r in 1 2; do for v in "0 0" "1 0" "1 16" "1 32"; do set -- $v
        timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream --service-pipeline $1 --service-split-min $2 > $O/svc_p$1_s$2_r$r.json 2> $O/svc_p$1_s$2_r$r.err || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    k2mall) timeout -k 10 400 python3 probes/k2_mall_probe.py 3 > $O/k2_mall.json 2> $O/k2_mall.err ;;
    gloo4) AIDFP_BENCH_BACKEND=gloo timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu > $O/gloo4.json 2> $O/gloo4.err ;;
    k6pmc)
      P="python3 probes/stream_host_profile.py --seconds 30"
      timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -T -d $O/k6pmc/sq -o run --output-format csv -- $P > $O/k6pmc_sq.txt 2> $O/k6pmc_sq.err &&
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d $O/k6pmc/fetch -o run --output-format csv -- $P > $O/k6pmc_fetch.txt 2> $O/k6pmc_fetch.err &&
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d $O/k6pmc/write -o run --output-format csv -- $P > $O/k6pmc_write.txt 2> $O/k6pmc_write.err ;;
    k6res)
      rc=0
      for r in 1 2; do for lib in product ${K6AB_VARIANTS:?set K6AB_VARIANTS}; do
        if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
        echo "== $lib $r" >> $O/k6res.txt
        env $L timeout -k 10 200 python3 bench_resample.py --no-cpu >> $O/k6res.txt 2>/dev/null || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    settleab)
      rc=0
      for r in 1 2 3; do for v in "20 0.1" "100 0.1" "100 0.5"; do set -- $v
        echo "== steps $1 settle $2 round $r" >> $O/settle_ab.txt
        timeout -k 10 200 python3 bench.py --steps $1 --settle $2 --no-cpu --no-fullband --no-catalog --no-service --no-stream > $O/settle_tmp.json 2>/dev/null || { rc=$?; break 2; }
        tail -1 $O/settle_tmp.json | cut -c1-220 >> $O/settle_ab.txt
      done; done
      [ $rc -eq 0 ] ;;
    k5ab)
      rc=0
      for r in 1 2; do for lib in product ${K5AB_VARIANTS:?set K5AB_VARIANTS}; do
        if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
        echo "== $lib $r" >> $O/k5ab.txt
        env $L timeout -k 10 400 python3 bench_match.py --no-cpu --category-queries 200 > $O/k5ab_tmp.json 2>/dev/null || { rc=$?; break 2; }
        tail -1 $O/k5ab_tmp.json >> $O/k5ab.txt
      done; done
      [ $rc -eq 0 ] ;;
    copyab)
      rc=0
      for r in 1 2 3; do for m in 4194304 2097152; do
        AIDFP_COPY_MIN_FLOATS=$m timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream > $O/svc_copy${m}_r$r.json 2> $O/svc_copy${m}_r$r.err || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    copythr)
      rc=0
      for r in 1 2 3; do for t in 4 8; do
        AIDFP_COPY_THREADS=$t timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream > $O/svc_thr${t}_r$r.json 2> $O/svc_thr${t}_r$r.err || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    winab)
      rc=0
      for r in 1 2 3; do for w in ${WINAB_MS:-0.5 0.2 1.0}; do
        timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream --service-window-ms $w > $O/svc_win${w}_r$r.json 2> $O/svc_win${w}_r$r.err || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    splitab)
      rc=0
      for r in 1 2 3; do for m in ${SPLITAB_MIN:-16 8 32}; do
        timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream --service-split-min $m > $O/svc_split${m}_r$r.json 2> $O/svc_split${m}_r$r.err || { rc=$?; break 2; }
      done; done
      [ $rc -eq 0 ] ;;
    svc)
      timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-fullband --no-catalog --no-stream > $O/svc.json 2> $O/svc.err ;;
    k6ab)
      rc=0
      for r in 1 2 3; do for lib in product ${K6AB_VARIANTS:?set K6AB_VARIANTS}; do
        if [ $lib = product ]; then L=""; else L="AIDFP_LIB=$GRAFT_REPO_ROOT/audio-ident_amd/build/$lib/libaidfp.so"; fi
        echo "== $lib $r" >> $O/k6ab.txt
        env $L timeout -k 10 200 python3 probes/stream_host_profile.py --seconds 30 --pipelined > $O/k6_${lib}_$r.txt 2>/dev/null || { rc=$?; break 2; }
        head -1 $O/k6_${lib}_$r.txt >> $O/k6ab.txt
      done; done
      [ $rc -eq 0 ] ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc"
  [ $rc -eq 0 ] || exit $((10 + i))
done
echo done
