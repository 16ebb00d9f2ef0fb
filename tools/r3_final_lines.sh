# Round-3 refresh of the per-config bench lines and the end-to-end pipeline lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
[ -n "${PIPE_ONLY:-}" ] || bash tools/bench_all.sh || exit 1
for args in "--frames 8" "--frames 32" "--frames 8 --torch-cnn" "--frames 8 --views"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python3 tools/bench_pipeline.py $args > gpurun_out/pipe_$tag.json 2> gpurun_out/pipe_$tag.err || { tail -5 gpurun_out/pipe_$tag.err; exit 1; }
  echo "pipeline $tag: $(tail -1 gpurun_out/pipe_$tag.json | cut -c1-200)"
done
