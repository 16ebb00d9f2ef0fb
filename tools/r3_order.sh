#!/bin/bash
# (Ran at commit 10edbe4 or earlier: the FVP_GATHER_ORDER / FVP_GATHER_TILE_X / FVP_GATHER_COLS /
# FVP_OTF_VOXELS knobs were removed once the A/B settled; check that commit out to reproduce.)
# Gather slot order A/B (FVP_GATHER_ORDER=col = z fastest, default = layer-major):
# the voxelize parity tests (every config bit-exact), then bench lines per order,
# interleaved, two repeats; and the C5 layout kernel A/B under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-ord}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_digests.py tests/test_gpu_columns.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for ord in col layer; do
    for wb in ${WORKLOADS:-c2:256 c4:64 c3:256 c5:8}; do
      w=${wb%%:*}; b=${wb##*:}
      FVP_GATHER_ORDER=$ord timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_${ord}_${w}_$rep.log 2>&1 || { tail -20 gpurun_out/${T}_${ord}_${w}_$rep.log; exit 1; }
      grep '^{' gpurun_out/${T}_${ord}_${w}_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$ord $w rep$rep', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'), d.get('latency_b1_graph_ms'), r.get('channels_last_input',{}).get('frac'))"
    done
  done
done
