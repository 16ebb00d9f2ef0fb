# Same-box A/B of an environment knob on bench lines: KNOB=NAME VALUES="a b" WORKLOADS="c2 c4" REPS=2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for w in ${WORKLOADS:-c2}; do
    for v in ${VALUES}; do
      env $KNOB=$v timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --traffic off --cpu-baseline off > gpurun_out/abenv_${v}_${w}_$r.log 2>&1 || { tail -20 gpurun_out/abenv_${v}_${w}_$r.log; exit 1; }
      grep '^{' gpurun_out/abenv_${v}_${w}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$KNOB=$v $w rep$r', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), d.get('latency_b1_graph_ms'), d.get('latency_b1_abi_ms'))"
    done
  done
done
