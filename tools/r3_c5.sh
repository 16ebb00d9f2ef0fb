# C5 / C4 / C2 bench lines (no CPU baseline / PMC) and the digest + full-size tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-c5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -q -m gpu --timeout 120 --timeout-method thread -x > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for w in ${WORKLOADS:-c5 c4 c2}; do
  timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-5} --warmup 2 --traffic off --cpu-baseline off > gpurun_out/${T}_bench_$w.log 2>&1 || { tail -20 gpurun_out/${T}_bench_$w.log; exit 1; }
  grep '^{' gpurun_out/${T}_bench_$w.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), d.get('latency_b1_graph_ms'))"
done
