#!/bin/bash
# Round-4 end-of-session refresh, part A: the full -m gpu suite, smoke, the default bench line
# (CPU baseline + traffic PMC) and its rocprofv3 kernel stats; the C3 B=8 step over 200 steps;
# the JLN line.  Part B (FINAL_B=1): one line per config with the CPU baseline + the pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/r4final; mkdir -p $O
if [ -z "${FINAL_B:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
  tail -1 $O/bench_c2.json | cut -c1-300
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --traffic off --cpu-baseline off > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
  python3 tools/kstats.py $O/prof_c2
  timeout -k 10 300 python bench.py --workload c3 --batch 8 --steps 200 --warmup 20 --traffic off --cpu-baseline off > $O/bench_c3_b8.json 2> $O/bench_c3_b8.err || { tail -20 $O/bench_c3_b8.err; exit 1; }
  tail -1 $O/bench_c3_b8.json | cut -c1-300
  timeout -k 10 300 python3 tools/bench_jln.py --frames 32 --steps 10 > $O/jln.json 2> $O/jln.err || { tail -20 $O/jln.err; exit 1; }
  tail -1 $O/jln.json | cut -c1-300
  echo "final A done"
else
  for wl in c1 c2 c3 c4 c5; do
    timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 2 --traffic off --cpu-baseline on > $O/all_$wl.json 2> $O/all_$wl.err || { tail -20 $O/all_$wl.err; exit 1; }
    echo "$wl: $(tail -1 $O/all_$wl.json | cut -c1-200)"
  done
  for wb in c4:32 c5:32; do
    w=${wb%%:*}; b=${wb##*:}
    timeout -k 10 300 python bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/all_${w}_b$b.json 2> $O/all_${w}_b$b.err || { tail -20 $O/all_${w}_b$b.err; exit 1; }
  done
  : > $O/pipeline.jsonl
  for extra in "" "--views"; do
    timeout -k 10 300 python3 tools/bench_pipeline.py $extra >> $O/pipeline.jsonl 2> $O/pipeline.err || { tail -20 $O/pipeline.err; exit 1; }
  done
  cat $O/pipeline.jsonl | cut -c1-300
  echo "final B done"
fi
