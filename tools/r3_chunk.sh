#!/bin/bash
# (Ran on a temporary build with an FVP_CHUNK_FRAMES knob.)  fp32 frames per chunk with layer-major slots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'))"; }
for rep in 1 2; do
  for wb in ${SWEEP:-c2:256:8 c2:256:4 c2:256:2 c2:256:12 c4:64:8 c4:64:4 c4:64:2}; do
    IFS=: read w b cf <<< "$wb"; L=gpurun_out/chunk_${w}_${cf}_$rep.log
    FVP_CHUNK_FRAMES=$cf timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
    line $L "$w chunk$cf rep$rep"
  done
done
