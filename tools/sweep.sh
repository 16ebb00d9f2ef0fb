#!/bin/bash
# bench sweep over env knobs; one line per setting
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in ${CHUNKS:-40}; do for pct in ${PCTS:-100}; do
  FVP_CHUNK_MB=$mb FVP_LAYOUT_PCT=$pct timeout -k 10 200 python bench.py --steps 10 --warmup 2 --traffic off --cpu-baseline off > gpurun_out/sweep_${mb}_${pct}.log 2>&1
  rc=$?; if [ $rc -ge 124 ]; then echo "stop rc=$rc"; exit $rc; fi
  echo "chunk_mb=$mb layout_pct=$pct $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep_${mb}_${pct}.log').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'])")"
done; done
