#!/bin/bash
# A/B of frames per fp16 pair-table entry (FVP_PAIR_FRAMES=2 vs 4) at C5, after
# the batch-invariance tests of both settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-pair4}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "frame_pairs" -q -m gpu --timeout 120 --timeout-method thread -x > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for nf in 2 4; do
    for b in ${BATCHES:-8 32}; do
      FVP_PAIR_FRAMES=$nf timeout -k 10 300 python3 bench.py --workload c5 --batch $b --steps ${STEPS:-5} --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_nf${nf}_b${b}_$rep.log 2>&1 || { tail -20 gpurun_out/${T}_nf${nf}_b${b}_$rep.log; exit 1; }
      grep '^{' gpurun_out/${T}_nf${nf}_b${b}_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('nf$nf b$b rep$rep', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'))"
    done
  done
done
