#!/bin/bash
# (Ran at commit 3524f68: the camera-outer kernel was reverted after this A/B.)
# PMC of the C2 gather: block gather (FVP_CAM_OUTER=0) vs camera-outer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
G="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU"
for co in 0 1; do
  FVP_CAM_OUTER=$co TAG=pmcco_$co PMC_GROUPS="$G" bash tools/pmc.sh > gpurun_out/pmcco_$co.txt 2>&1 || { tail -20 gpurun_out/pmcco_$co.txt; exit 1; }
  echo "== co$co"; grep -A16 "voxelize_co_kernel\|voxelize_kernel" gpurun_out/pmcco_$co.txt | head -34
done
