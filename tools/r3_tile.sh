#!/bin/bash
# (Ran at commit 10edbe4 or earlier: the FVP_GATHER_ORDER / FVP_GATHER_TILE_X / FVP_GATHER_COLS /
# FVP_OTF_VOXELS knobs were removed once the A/B settled; check that commit out to reproduce.)
# Column-tile A/B (FVP_GATHER_TILE_X=1: 1 x cols x-row strips; 2: 2 x cols/2 tiles),
# both with layer-major slots; C4 also at 8 columns (FVP_GATHER_COLS=8).  Full GPU
# test suite first (the default tiling), then interleaved bench lines, two repeats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-tile}
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
fi
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'), d.get('latency_b1_graph_ms'), r.get('channels_last_input',{}).get('frac'))"; }
for rep in 1 2; do
  for txv in 1 2; do
    for wb in ${WORKLOADS:-c2:256 c3:256 c4:64 c5:8}; do
      w=${wb%%:*}; b=${wb##*:}; L=gpurun_out/${T}_tx${txv}_${w}_$rep.log
      FVP_GATHER_TILE_X=$txv timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
      line $L "tx$txv $w rep$rep"
    done
    L=gpurun_out/${T}_tx${txv}_c4c8_$rep.log
    FVP_GATHER_COLS=8 FVP_GATHER_TILE_X=$txv timeout -k 10 300 python3 bench.py --workload c4 --batch 64 --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
    line $L "tx$txv c4-cols8 rep$rep"
  done
done
