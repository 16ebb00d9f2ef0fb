#!/bin/bash
# (Ran at commit 10edbe4 or earlier: the FVP_GATHER_ORDER / FVP_GATHER_TILE_X / FVP_GATHER_COLS /
# FVP_OTF_VOXELS knobs were removed once the A/B settled; check that commit out to reproduce.)
# C5 (on the fly, 4 frames per entry): voxels per block 128 (default) vs 256 vs 64, layer-major slots.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'))"; }
for rep in 1 2; do
  for vx in 128 256 64; do
    L=gpurun_out/otfvox_${vx}_$rep.log
    FVP_OTF_VOXELS=$vx timeout -k 10 300 python3 bench.py --workload c5 --batch 8 --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
    line $L "c5 vox$vx rep$rep"
  done
done
