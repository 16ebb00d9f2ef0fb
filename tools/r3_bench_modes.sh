# bench.py modes other than the default line: channels-last input, C1, x-slabs, a 2-rank gloo rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
run() {  # name args...
  local n=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/modes_$n.log 2>&1 || { echo "$n FAILED"; tail -20 gpurun_out/modes_$n.log; exit 1; }
  grep '^{' gpurun_out/modes_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['n_gpus'], d['config'].get('parallelism'), d.get('latency_b1_abi_ms'))"
}
run cl python3 bench.py --heatmap-layout channels-last --steps 5 --traffic off --cpu-baseline off
run c1 python3 bench.py --workload c1 --steps 5 --traffic off --cpu-baseline off
run slabs python3 bench.py --workload c5 --slabs --batch 4 --steps 3 --traffic off --cpu-baseline off
run gloo2 env FVP_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --traffic off --cpu-baseline off
