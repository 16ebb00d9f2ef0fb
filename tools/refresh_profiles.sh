# One GPU session refreshing every profiles/ line: bench lines C1..C5 (+ SURVEY
# batch sizes), the JLN line, the CNN line and the end-to-end pipeline, plus
# a rocprofv3 kernel-trace summary of the JLN line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TRAFFIC=${TRAFFIC:-off} bash tools/bench_all.sh || exit $?
timeout -k 10 300 python tools/bench_cnn.py > gpurun_out/all_cnn.log 2>&1; echo "cnn rc=$?"
timeout -k 10 300 python tools/bench_pipeline.py > gpurun_out/all_pipeline.log 2>&1; echo "pipeline rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jln -o run -- python3 tools/bench_jln.py --frames 32 > gpurun_out/prof_jln.log 2>&1; echo "jln prof rc=$?"
