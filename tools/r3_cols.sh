#!/bin/bash
# (Ran at commit 10edbe4 or earlier: the FVP_GATHER_ORDER / FVP_GATHER_TILE_X / FVP_GATHER_COLS /
# FVP_OTF_VOXELS knobs were removed once the A/B settled; check that commit out to reproduce.)
# Columns per cached-grid block with layer-major slots (FVP_GATHER_COLS sweep), C2 / C3 / C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-cols}
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'), r.get('channels_last_input',{}).get('frac'))"; }
for rep in 1 2; do
  for wb in c2:256:4 c2:256:8 c2:256:16 c3:256:8 c3:256:16 c4:64:4 c4:64:8 c4:64:16; do
    IFS=: read w b cols <<< "$wb"; L=gpurun_out/${T}_${w}_c${cols}_$rep.log
    FVP_GATHER_COLS=$cols timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
    line $L "$w cols$cols rep$rep"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_c2 -o run -- python3 bench.py --workload c2 --steps 10 --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_prof_c2.log 2>&1 || { tail -20 gpurun_out/${T}_prof_c2.log; exit 1; }
f=$(find gpurun_out/${T}_prof_c2 -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | cut -c1-160 | head -12
