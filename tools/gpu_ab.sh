# GPU tests, then rocprofv3 kernel stats of bench.py under two settings of an
# env knob.  usage: KNOB=FVP_TAP_ROWS VALUES="0 1" WL=c2 bash tools/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for wl in ${WL:-c2}; do
for val in ${VALUES:-0 1}; do
  export ${KNOB:-FVP_TAP_ROWS}=$val
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${wl}_$val -o run -- python3 bench.py --workload $wl --steps 10 --warmup 2 --traffic off --cpu-baseline off ${BENCH_ARGS:-} > gpurun_out/prof_${wl}_$val.log 2>&1
  rc=$?; echo "$wl $val rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
done
exit 0
