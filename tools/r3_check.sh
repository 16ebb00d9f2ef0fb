#!/bin/bash
# Full GPU test suite, then bench lines (no CPU baseline / PMC) for $WORKLOADS
# ("c5:8 c5:32 c2" = workload:batch) -- one call's round-trip check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-chk}
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
  tail -1 gpurun_out/${T}_tests.log
fi
for wb in ${WORKLOADS:-c5:8 c5:32 c2:256}; do
  w=${wb%%:*}; b=${wb##*:}
  timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps ${STEPS:-10} --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_bench_${w}_b$b.log 2>&1 || { tail -20 gpurun_out/${T}_bench_${w}_b$b.log; exit 1; }
  grep '^{' gpurun_out/${T}_bench_${w}_b$b.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$w b$b', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'), d.get('latency_b1_graph_ms'))"
done
