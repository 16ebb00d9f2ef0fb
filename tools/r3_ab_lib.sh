# Same-box A/B of two libfvp builds on bench lines: LIBS="a.so b.so" WORKLOADS="c5 c2" REPS=2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for w in ${WORKLOADS:-c5 c4 c2}; do
    for lib in ${LIBS}; do
      n=$(basename $lib .so)
      FVP_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $w --steps ${STEPS:-5} --warmup 2 --traffic off --cpu-baseline off > gpurun_out/ab_${n}_${w}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${n}_${w}_$r.log; exit 1; }
      grep '^{' gpurun_out/ab_${n}_${w}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n $w rep$r', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), d.get('latency_b1_graph_ms'))"
    done
  done
done
