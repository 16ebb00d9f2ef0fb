# rocprofv3 kernel stats of bench.py for each VALUE of an env knob and each workload (A/B/C...).
# usage: KNOB=FVP_BAND VALUES="0 8 16" WL="c2 c5" bash tools/ab_multi.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for wl in ${WL:-c2}; do
for val in ${VALUES:-0 1}; do
  export ${KNOB}=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_$val -o run -- python3 bench.py --workload $wl --steps 10 --warmup 2 --traffic off --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/prof_${wl}_$val.log 2>&1
  rc=$?; echo "$wl $val rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
