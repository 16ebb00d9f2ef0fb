#!/bin/bash
# Round-2 PMC evidence: per-kernel HBM bytes (FETCH_SIZE / WRITE_SIZE, separate
# passes), L2 hit/miss and the texture-path counters (TA/TD busy and stall) of
# the default C2 workload (planar and channels-last input) and of C5, plus
# rocprofv3 kernel stats of each.  Summaries by tools/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
GROUPS_ALL="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
GRBM_GUI_ACTIVE GRBM_COUNT"
for cfg in "c2:" "c2cl:--heatmap-layout channels-last" "c5:--workload c5"; do
  tag=${cfg%%:*}; extra=${cfg#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2prof_$tag -o run -- \
    python3 bench.py --traffic off --cpu-baseline off --steps 10 --warmup 2 $extra > gpurun_out/r2prof_$tag.log 2>&1
  rc=$?; echo "prof $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
  TAG=r2pmc_$tag PMC_GROUPS="$GROUPS_ALL" BENCH_EXTRA="$extra" bash tools/pmc.sh > gpurun_out/r2pmc_$tag.txt 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
