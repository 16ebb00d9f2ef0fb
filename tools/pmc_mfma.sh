#!/bin/bash
# MFMA utilisation evidence: SQ_VALU_MFMA_BUSY_CYCLES (summed over SIMDs) and
# GRBM_GUI_ACTIVE (summed over XCDs) per conv kernel of the bf16 / fp32
# ResNet-50 backbone.
# Utilisation = MFMA_BUSY / (SIMDs x GRBM_GUI_ACTIVE / XCDs); summaries by tools/pmc_db.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(dirname "$0")/..}; O=$R/gpurun_out/pmc_mfma; rm -rf $O; mkdir -p $O
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --pmc $P -d $O/bb_bf16 -o run -- python3 $R/tools/backbone_layers.py --bf16 > /dev/null || exit $?
timeout -s KILL 240 rocprofv3 --pmc $P -d $O/bb_f32 -o run -- python3 $R/tools/backbone_layers.py > /dev/null || exit $?
for d in bb_bf16 bb_f32; do python3 $R/tools/pmc_db.py --match conv $O/$d > $O/$d.txt || exit $?; rm -rf $O/$d; done
echo done
