#!/bin/bash
# After an fp32 conv change: pipeline lines, backbone / CNN benches, fp32
# backbone layers and the fp32 MFMA-utilisation PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash tools/refresh_pipeline.sh || exit $?
timeout -k 10 200 python3 tools/backbone_layers.py > gpurun_out/backbone_layers_f32.json 2>/dev/null || exit $?
timeout -k 10 300 python3 tools/bench_backbone.py > gpurun_out/bench_backbone.json 2>/dev/null || exit $?
timeout -k 10 200 python3 tools/bench_cnn.py > gpurun_out/bench_cnn.json 2>/dev/null || exit $?
R=$PWD; O=$R/gpurun_out/pmc_mfma; mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
   -d $O/bb_f32 -o run -- python3 $R/tools/backbone_layers.py > /dev/null) || exit $?
python3 tools/pmc_db.py --match conv $O/bb_f32 > $O/bb_f32.txt || exit $?
rm -rf $O/bb_f32
echo done
