#!/bin/bash
# pairs_rows_kernel vs the per-entry pair-table layout (FVP_PAIRS_LAYOUT=entry):
# the fp16 parity tests, then rocprofv3 kernel stats of C5 B=8 bench steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-pl}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_digests.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for mode in rows entry; do
  FVP_PAIRS_LAYOUT=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_$mode -o run -- python3 bench.py --workload c5 --batch 8 --steps 10 --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_bench_$mode.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$mode.log; exit 1; }
  grep '^{' gpurun_out/${T}_bench_$mode.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$mode', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'))"
  f=$(find gpurun_out/${T}_prof_$mode -name '*kernel_stats.csv' | head -1); grep -i "pairs\|voxelize" "$f" | cut -d, -f1-4 | cut -c1-200
done
