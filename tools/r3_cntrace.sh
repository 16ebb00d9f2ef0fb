# CenterNet (C3 B=8) kernel durations per fp32 kernel choice, from rocprofv3 kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for a in ${ALGOS:-auto halo pertap nosplit dma}; do
  rm -rf gpurun_out/cntr${TAG:-}_$a
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cntr${TAG:-}_$a -o run -- \
    python3 tools/cnn_trace.py run --net centernet --images ${IMAGES:-8} --algo $a > gpurun_out/cntr${TAG:-}_$a.log 2>&1 || exit 1
  python3 tools/cnn_trace.py parse gpurun_out/cntr${TAG:-}_$a > gpurun_out/cntr${TAG:-}_$a.json || exit 1
  echo "$a $(python3 -c "import json;d=json.load(open('gpurun_out/cntr${TAG:-}_$a.json'));print(d['last_busy_us'],d['last_span_us'],d['min_span_us'],d['dispatches'])")"
done
