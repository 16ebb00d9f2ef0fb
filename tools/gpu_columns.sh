# GPU: the recomputed-columns tests, then the heatmaps -> poses pipeline with and without the cube
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_columns.py tests/test_integration.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/col_tests.log 2>&1 || { tail -40 gpurun_out/col_tests.log; exit 1; }
tail -1 gpurun_out/col_tests.log
: > gpurun_out/col_pipe.jsonl
for f in 8 32; do for r in 0 1; do for v in "" "--bf16"; do
  FVP_RECOMPUTE_COLUMNS=$r timeout -k 10 200 python tools/bench_pipeline.py --frames $f --steps 40 $v 2>/dev/null | grep "^{" | sed "s/^{/{\"recompute\": $r, \"frames\": $f, \"args\": \"$v\", /" >> gpurun_out/col_pipe.jsonl || exit 1
done; done; done
python -c "
import json
for l in open('gpurun_out/col_pipe.jsonl'):
    d=json.loads(l); print(d['recompute'], d['frames'], d['args'], d['value'])"
FVP_RECOMPUTE_COLUMNS=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/col_prof -o run -- python3 tools/bench_pipeline.py --frames 8 --steps 40 > gpurun_out/col_prof.log 2>&1; echo prof rc=$?
