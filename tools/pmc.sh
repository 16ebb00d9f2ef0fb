#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains) over a
# short bench run; summarised per kernel by tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  # PMC_CMD: the program to profile (default: a short bench run)
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d $OUT/p$i -o run -- \
    ${PMC_CMD:-python3 bench.py --child --steps 3 --warmup 1 --traffic off --cpu-baseline off ${BENCH_EXTRA:-}} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($group) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<< "${PMC_GROUPS:-TCC_HIT_sum TCC_MISS_sum
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES}"
python3 tools/pmc_summary.py $OUT
if [ -n "${PMC_CLEAN:-}" ]; then rm -rf $OUT/p*/; fi
