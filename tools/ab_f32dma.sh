#!/bin/bash
# fp32 LDS-DMA conv kernel A/B (FVP_F32_DMA=1 vs 0): backbone layers, CNN
# nets, views -> poses pipeline.  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/f32dma
mkdir -p $O
for d in 1 0; do
  export FVP_F32_DMA=$d
  timeout -k 10 120 python tools/backbone_layers.py > $O/bb_layers_$d.json 2> $O/err_$d.log || exit $?
  timeout -k 10 120 python tools/cnn_layers.py --net p2p > $O/p2p_$d.json 2>> $O/err_$d.log || exit $?
  timeout -k 10 120 python tools/cnn_layers.py --net centernet > $O/cn_$d.json 2>> $O/err_$d.log || exit $?
  timeout -k 10 200 python tools/bench_cnn.py > $O/bench_cnn_$d.json 2>> $O/err_$d.log || exit $?
  timeout -k 10 200 python tools/bench_pipeline.py --views --workload c3 > $O/pipe_views_$d.json 2>> $O/err_$d.log || exit $?
  timeout -k 10 200 python tools/bench_pipeline.py --workload c3 > $O/pipe_$d.json 2>> $O/err_$d.log || exit $?
done
