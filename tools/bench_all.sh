#!/bin/bash
# One bench line per BASELINE config (C1..C5) + the SURVEY §8(d) batch sizes + the JLN line
# (CPU=on adds the CPU baseline to each line; the default headline run has it).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag args... (STEPS / WARMUP: per-call overrides)
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps ${STEPS:-10} --warmup ${WARMUP:-2} --traffic ${TRAFFIC:-off} \
    --cpu-baseline ${CPU:-off} > gpurun_out/all_$tag.log 2>&1
  local rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
}
for wl in ${WORKLOADS:-c1 c2 c3 c4 c5}; do run $wl --workload $wl; done
if [ -z "${NO_BATCHES:-}" ]; then
  STEPS=200 WARMUP=20 run c3_b8 --workload c3 --batch 8  # 0.13 ms steps: enough of them
  run c4_b32 --workload c4 --batch 32
  run c5_b32 --workload c5 --batch 32
fi
timeout -k 10 300 python tools/bench_jln.py --frames 32 > gpurun_out/all_jln.log 2>&1; echo "jln rc=$?"
