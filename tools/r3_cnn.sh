# CenterNet per-layer times at C3 B=8 (80x80) under each fp32 kernel choice, and the CNN bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for a in auto dma halo pertap; do
  timeout -k 10 120 python3 tools/cnn_layers.py --net centernet --images 8 --algo $a > gpurun_out/r3_cn_$a.json 2> gpurun_out/r3_cn_$a.err || exit 1
done
timeout -k 10 200 python3 tools/bench_cnn.py > gpurun_out/r3_bench_cnn.json 2> gpurun_out/r3_bench_cnn.err || exit 1
echo ok
