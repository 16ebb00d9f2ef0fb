#!/bin/bash
# One gpurun session on one MI355X: the steps named on the command line, in order, each under its
# own time limit; the first failing step ends the session.  Output under gpurun_out/$OUT (default s).
#   tests   the -m gpu suite            smoke  __graft_entry__.smoke()
#   bench   the default bench line (CPU baseline + traffic PMC; the PMC CSVs copied to $O/bench_pmc)
#   prof    rocprofv3 kernel trace of the default bench + per-launch-shape summary
#   c3b8    bench.py --workload c3 --batch 8 over 200 steps (c3b8g: the same replayed from hipGraphs)
#   jln     tools/bench_jln.py (32 frames)
#   all     one bench line per config (C1-C5, C4/C5 at B=32)
#   pipe    tools/bench_pipeline.py (heatmaps -> poses, and views)
#   gloo2   bench.py --gpus 2 over gloo on the one GPU (a rehearsal of the N-rank launch)
#   ab      for each library ab_libs/<name>.so in $AB_LIBS (tools/ab_build.sh), REPEAT (2) rounds of:
#           a bench line (no traffic / CPU baseline) + a kernel trace with its launch shapes
#   step    tools/step_host.py (host / GPU time per part of the small-batch step; $STEP_ARGS)
#   overlap tools/overlap_probe2.py for each library in $AB_LIBS
#   pmcl2   TCC_HIT / TCC_MISS (one counter pass each) of a short bench run per library in $AB_LIBS
#   c2c     tools/c2c_probe.py at Z = 20 / 32 / 64 (one-launch C2CNet vs per-layer kernels)
#   pipe5   tools/bench_pipeline.py at C5 (8 frames: the HDN with Z = 64 columns)
#   pipetrace rocprofv3 kernel stats of tools/bench_pipeline.py (heatmaps -> poses, C3 B = 8)
#   pmcfwd  tools/pmc_forwards.sh (MFMA busy / ops of the shipped CNN forwards)
#   nmsp    tools/nms_probe.py (NMS top-K [+ columns] per launch, smooth and plateau maps)
#   wino    tools/wino_probe.py (Winograd vs direct 3x3 layers)
#   cnn     tools/bench_cnn.py
#   cntrace rocprofv3 kernel trace of one CenterNet (8 frames) and one P2PNet (240 images) forward, per dispatch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${OUT:-s}; mkdir -p $O
fail() { echo "FAILED: $1"; tail -40 "$2"; exit 1; }
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/gpu_tests.log 2>&1 || fail tests $O/gpu_tests.log
           tail -1 $O/gpu_tests.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
           tail -1 $O/smoke.log ;;
    bench) rm -rf gpurun_out/bench_pmc
           timeout -k 10 600 python bench.py $BENCH_ARGS > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
           if [ -d gpurun_out/bench_pmc ]; then mkdir -p $O/bench_pmc && cp -r gpurun_out/bench_pmc/. $O/bench_pmc/; fi
           cut -c1-400 $O/bench.json ;;
    prof)  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --traffic off --cpu-baseline off $BENCH_ARGS > $O/prof.log 2>&1 || fail prof $O/prof.log
           python3 tools/launch_shapes.py $O/prof --csv $O/launch_shapes.csv --top 8 ;;
    c3b8)  timeout -k 10 300 python bench.py --workload c3 --batch 8 --steps 200 --warmup 20 --traffic off --cpu-baseline off > $O/bench_c3_b8.json 2> $O/bench_c3_b8.err || fail c3b8 $O/bench_c3_b8.err
           cut -c1-300 $O/bench_c3_b8.json ;;
    c3b8g) timeout -k 10 300 python bench.py --workload c3 --batch 8 --steps 200 --warmup 20 --graph on --traffic off --cpu-baseline off > $O/bench_c3_b8_graph.json 2> $O/bench_c3_b8_graph.err || fail c3b8g $O/bench_c3_b8_graph.err
           cut -c1-300 $O/bench_c3_b8_graph.json ;;
    jln)   timeout -k 10 300 python3 tools/bench_jln.py --frames 32 --steps 10 > $O/jln.json 2> $O/jln.err || fail jln $O/jln.err
           cut -c1-300 $O/jln.json ;;
    all)   for wl in c1 c2 c3 c4 c5; do
             tr=off; case $wl in c4|c5) tr=auto;; esac  # (C4 / C5: the FETCH / WRITE counters too)
             timeout -k 10 600 python bench.py --workload $wl --steps 10 --warmup 2 --traffic $tr --cpu-baseline on > $O/all_$wl.json 2> $O/all_$wl.err || fail all_$wl $O/all_$wl.err
             echo "$wl: $(cut -c1-200 $O/all_$wl.json)"
           done
           for wb in c4:32 c5:32; do
             w=${wb%%:*}; b=${wb##*:}
             timeout -k 10 300 python bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/all_${w}_b$b.json 2> $O/all_${w}_b$b.err || fail all_${w}_b$b $O/all_${w}_b$b.err
           done ;;
    pipe)  : > $O/pipeline.jsonl
           for extra in "" "--views"; do
             timeout -k 10 300 python3 tools/bench_pipeline.py $extra >> $O/pipeline.jsonl 2> $O/pipeline.err || fail pipe $O/pipeline.err
           done
           cut -c1-300 $O/pipeline.jsonl ;;
    gloo2) FVP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/bench_gloo2.json 2> $O/bench_gloo2.err || fail gloo2 $O/bench_gloo2.err
           cut -c1-400 $O/bench_gloo2.json ;;
    ab)    for rep in $(seq 1 ${REPEAT:-2}); do
             for lib in $AB_LIBS; do
               FVP_LIB=ab_libs/$lib.so timeout -k 10 300 python bench.py --traffic off --cpu-baseline off $BENCH_ARGS > $O/ab_${lib}_$rep.json 2> $O/ab_${lib}_$rep.err || fail ab_$lib $O/ab_${lib}_$rep.err
               echo "$lib $rep: $(python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).readlines()[-1]); r=b['roofline']; print(b['value'], r['kernel_ms'], r['frac'], r.get('channels_last_input',{}).get('frac'))" $O/ab_${lib}_$rep.json)"
               if [ "$rep" = 1 ]; then
                 FVP_LIB=ab_libs/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/abprof_$lib -o run -- python3 bench.py --traffic off --cpu-baseline off $BENCH_ARGS > $O/abprof_$lib.log 2>&1 || fail abprof_$lib $O/abprof_$lib.log
                 python3 tools/launch_shapes.py $O/abprof_$lib --csv $O/abprof_$lib.csv --top 4
               fi
             done
           done ;;
    step)  timeout -k 10 300 python3 tools/step_host.py $STEP_ARGS > $O/step.json 2> $O/step.err || fail step $O/step.err
           cat $O/step.json ;;
    overlap) for lib in $AB_LIBS; do
             FVP_LIB=ab_libs/$lib.so timeout -k 10 300 python3 tools/overlap_probe2.py $OVERLAP_ARGS > $O/overlap_$lib.jsonl 2> $O/overlap_$lib.err || fail overlap_$lib $O/overlap_$lib.err
             cat $O/overlap_$lib.jsonl
           done ;;
    pmcl2) for lib in $AB_LIBS; do
             for c in TCC_HIT_sum TCC_MISS_sum; do
               FVP_LIB=ab_libs/$lib.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${lib}_$c -o run -- python3 bench.py --traffic off --cpu-baseline off --steps 3 --warmup 1 $BENCH_ARGS > $O/pmc_${lib}_$c.log 2>&1 || fail pmc_${lib}_$c $O/pmc_${lib}_$c.log
             done
           done
           python3 tools/pmc_kernels.py $O/pmc_* ;;
    c2c)   : > $O/c2c.jsonl
           for L in 20 32 64; do
             timeout -k 10 120 python3 tools/c2c_probe.py --L $L >> $O/c2c.jsonl 2> $O/c2c.err || fail c2c $O/c2c.err
           done
           cat $O/c2c.jsonl ;;
    pipe5) timeout -k 10 300 python3 tools/bench_pipeline.py --workload c5 --frames 8 --steps 5 > $O/pipeline_c5.jsonl 2> $O/pipeline_c5.err || fail pipe5 $O/pipeline_c5.err
           cut -c1-400 $O/pipeline_c5.jsonl ;;
    pipetrace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pipetrace -o run -- python3 tools/bench_pipeline.py --steps 5 > $O/pipetrace.log 2>&1 || fail pipetrace $O/pipetrace.log
           python3 -c "
import csv,sys
r=list(csv.DictReader(open('$O/pipetrace/run_kernel_stats.csv')))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:30]: print(f\"{x['Name'][:80]:80s} {x['Calls']:>6s} {float(x['AverageNs'])/1e3:9.1f} us {float(x['Percentage']):6.2f} %\")
" | tee $O/pipetrace_top.txt ;;
    pmcfwd) OUT=$OUT/pmcfwd timeout -k 10 1200 bash tools/pmc_forwards.sh || fail pmcfwd /dev/null ;;
    nmsp)  timeout -k 10 300 python3 tools/nms_probe.py > $O/nms_probe.json 2> $O/nms_probe.err || fail nmsp $O/nms_probe.err
           cat $O/nms_probe.json ;;
    wino)  timeout -k 10 300 python3 tools/wino_probe.py > $O/wino.jsonl 2> $O/wino.err || fail wino $O/wino.err
           cat $O/wino.jsonl ;;
    winoab) for lib in $AB_LIBS; do
             FVP_LIB=ab_libs/$lib.so timeout -k 10 300 python3 tools/wino_probe.py $WINO_ARGS > $O/wino_$lib.jsonl 2> $O/wino_$lib.err || fail wino_$lib $O/wino_$lib.err
             echo "== $lib"; python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(f\"{d['layer']:24s} direct {d['direct']['us']:8.1f} wino {d['wino']['us']:8.1f} x{d['speedup']:.2f} err {d['wino']['err']:.2e}\")
" $O/wino_$lib.jsonl
           done ;;
    cnn)   timeout -k 10 300 python3 tools/bench_cnn.py ${PMCDIR:+--pmc-dir $PMCDIR} $( [ -z "${PMCDIR:-}" ] && [ -d $O/pmcfwd ] && echo --pmc-dir $O/pmcfwd ) > $O/cnn.jsonl 2> $O/cnn.err || fail cnn $O/cnn.err
           cut -c1-400 $O/cnn.jsonl ;;
    cntrace) for nt in centernet:8 p2p:240; do
             net=${nt%%:*}; im=${nt##*:}
             timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$net -o run -- python3 tools/cnn_trace.py run --net $net --images $im --algo auto > $O/trace_$net.log 2>&1 || fail trace_$net $O/trace_$net.log
             python3 tools/cnn_trace.py parse $O/trace_$net > $O/trace_$net.json || fail parse_$net $O/trace_$net.json
             python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['last_busy_us'], d['last_span_us'], d['dispatches']); [print('  %7.2f %s' % (t, k[:90])) for t, k in d['kernels']]" $O/trace_$net.json $net
           done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session done $(date +%T)"
