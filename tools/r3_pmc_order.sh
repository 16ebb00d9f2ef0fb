#!/bin/bash
# (Ran at commit 10edbe4 or earlier: the FVP_GATHER_ORDER / FVP_GATHER_TILE_X / FVP_GATHER_COLS /
# FVP_OTF_VOXELS knobs were removed once the A/B settled; check that commit out to reproduce.)
# Per-kernel PMC of the C2 gather for the slot-order / tile variants (col strips, layer strips, layer 2x4 tiles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
G="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum"
for v in col:1 layer:1 layer:2; do
  o=${v%%:*}; t=${v##*:}
  FVP_GATHER_ORDER=$o FVP_GATHER_TILE_X=$t TAG=pmco_${o}_$t PMC_GROUPS="$G" bash tools/pmc.sh > gpurun_out/pmco_${o}_$t.txt 2>&1 || { tail -20 gpurun_out/pmco_${o}_$t.txt; exit 1; }
  echo "== $o tx$t"; grep -A30 "voxelize_kernel" gpurun_out/pmco_${o}_$t.txt | head -24
done
