#!/bin/bash
# One bench line per BASELINE config (C1..C5) + the JLN line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WORKLOADS:-c1 c2 c3 c4 c5}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --traffic ${TRAFFIC:-off} --cpu-seconds ${CPU_S:-5} > gpurun_out/all_$wl.log 2>&1
  rc=$?; echo "$wl rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
timeout -k 10 300 python tools/bench_jln.py --frames 32 > gpurun_out/all_jln.log 2>&1; echo "jln rc=$?"
