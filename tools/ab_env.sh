#!/bin/bash
# A/B of environment settings on one bench workload (experiments):
#   CFGS="FVP_NF=1 FVP_NF=2,OTHER=3" BENCH_ARGS="--workload c5" bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
: > gpurun_out/ab_env.txt
for cfg in ${CFGS:-none}; do
  ( export ${cfg//,/ } 2>/dev/null
    timeout -k 10 120 python3 bench.py --traffic off --cpu-baseline off --steps ${STEPS_N:-10} ${BENCH_ARGS:-} > gpurun_out/ab_tmp.json 2>/dev/null ) || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_tmp.json')); r=d['roofline']; print('$cfg', d['value'], r['kernel_ms'], r['frac'], r['tap_rate']['frac'])" >> gpurun_out/ab_env.txt
done
cat gpurun_out/ab_env.txt
