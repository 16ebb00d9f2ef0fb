#!/bin/bash
# (Ran at commit 3524f68: the camera-outer kernel was reverted after this A/B.)
# Camera-outer gather (voxelize_co_kernel) A/B: FVP_CAM_OUTER=0 (block gather) vs default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-co}
timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "digest or full_size or batch or whole or c2 or C2" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r.get('kernel_ms'), r.get('channels_last_input',{}).get('frac'))"; }
for rep in 1 2; do
  for co in 0 1; do
    for wb in ${WORKLOADS:-c2:256 c3:256}; do
      w=${wb%%:*}; b=${wb##*:}; L=gpurun_out/${T}_co${co}_${w}_$rep.log
      FVP_CAM_OUTER=$co timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $L 2>&1 || { tail -20 $L; exit 1; }
      line $L "co$co $w rep$rep"
    done
  done
done
