# B=1 latency (+ kernel stats) and the default C2 bench line on the current tree
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-ab}
mkdir -p gpurun_out
timeout -k 10 120 python tools/latency_b1.py > gpurun_out/${T}_lat.log 2>&1 && tail -1 gpurun_out/${T}_lat.log || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 tools/latency_b1.py > gpurun_out/${T}_prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --traffic off --cpu-baseline off > gpurun_out/${T}_bench.log 2>&1 || exit 1
grep '^{' gpurun_out/${T}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('bench', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['latency_b1_ms'], d['latency_b1_graph_ms'])"
