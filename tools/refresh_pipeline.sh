#!/bin/bash
# Views -> poses and heatmaps -> poses pipeline lines (fvp fp32, torch CNNs,
# fvp bf16), appended to gpurun_out/bench_pipeline.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
out=gpurun_out/bench_pipeline.jsonl; : > $out
for extra in "--views" "--views --torch-cnn" "--views --bf16" "" "--torch-cnn" "--bf16"; do
  timeout -k 10 300 python3 tools/bench_pipeline.py $extra >> $out 2>gpurun_out/pipeline.err || exit $?
  echo "pipeline $extra done"
done
