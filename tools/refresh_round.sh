# Refresh every profiles/round1 artefact in one GPU call: GPU tests, the
# default bench line (traffic PMC + CPU baseline) with its rocprofv3 kernel
# stats, every config's bench line, the JLN / CNN / pipeline lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/r_pytest.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/final_bench.sh || exit $?
NO_BATCHES= bash tools/bench_all.sh || exit $?
timeout -k 10 300 python tools/bench_cnn.py > gpurun_out/all_cnn.log 2>&1; echo "cnn rc=$?"
: > gpurun_out/all_pipeline.jsonl
for f in 8 32; do for v in "" "--torch-cnn" "--bf16"; do
  timeout -k 10 200 python tools/bench_pipeline.py --frames $f --steps 40 $v 2>/dev/null | grep "^{" >> gpurun_out/all_pipeline.jsonl || exit 1
done; done; echo "pipeline ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jln -o run -- python3 tools/bench_jln.py --frames 32 > gpurun_out/prof_jln.log 2>&1; echo "jln prof rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pipe -o run -- python3 tools/bench_pipeline.py --frames 8 --steps 40 > gpurun_out/prof_pipe.log 2>&1; echo "pipeline prof rc=$?"
