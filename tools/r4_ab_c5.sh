#!/bin/bash
# Same-box A/B of libfvp builds on bench lines + rocprof kernel stats:
#   LIBS="ab_libs/a.so ab_libs/b.so" WL="c5:8 c5:32" REPS=2 bash tools/r4_ab_c5.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/ab_${TAG:-c5}; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for wb in ${WL:-c5:8}; do
    w=${wb%%:*}; b=${wb##*:}
    for lib in ${LIBS}; do
      n=$(basename $lib .so)
      FVP_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $w --batch $b --steps ${STEPS:-10} --warmup 2 --traffic off --cpu-baseline off ${EXTRA:-} > $O/${n}_${w}_b${b}_$r.log 2>&1 || { tail -20 $O/${n}_${w}_b${b}_$r.log; exit 1; }
      grep '^{' $O/${n}_${w}_b${b}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n $w b$b rep$r', d['value'], d['ms_per_step'], r['frac'], r.get('tap_rate',{}).get('frac'), r['kernel_ms'])"
    done
  done
done
if [ -n "${KSTATS:-}" ]; then
  for lib in ${LIBS}; do
    n=$(basename $lib .so); w=${KSTATS%%:*}; b=${KSTATS##*:}
    FVP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks_$n -o run -- python3 bench.py --workload $w --batch $b --steps 10 --warmup 2 --traffic off --cpu-baseline off > $O/ks_$n.log 2>&1 || { tail -5 $O/ks_$n.log; exit 1; }
    python3 tools/kstats.py $O/ks_$n
  done
fi
