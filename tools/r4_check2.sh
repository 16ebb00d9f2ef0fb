#!/bin/bash
# Closing check after the 8-entry pair layout: the -m gpu suite, smoke, the default bench line, and
# the C5 lines (B = 8 with the CPU baseline, B = 32) with C5 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/r4check2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --traffic off --cpu-baseline off > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
tail -1 $O/bench_c2.json | cut -c1-250
timeout -k 10 400 python bench.py --workload c5 --steps 10 --warmup 2 --traffic off --cpu-baseline on > $O/all_c5.json 2> $O/all_c5.err || { tail -20 $O/all_c5.err; exit 1; }
tail -1 $O/all_c5.json | cut -c1-250
timeout -k 10 300 python bench.py --workload c5 --batch 32 --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/all_c5_b32.json 2> $O/all_c5_b32.err || { tail -20 $O/all_c5_b32.err; exit 1; }
tail -1 $O/all_c5_b32.json | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/prof_c5.log 2>&1 || { tail -20 $O/prof_c5.log; exit 1; }
python3 tools/kstats.py $O/prof_c5
echo "check2 done"
