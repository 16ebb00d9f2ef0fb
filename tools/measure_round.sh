#!/bin/bash
# One GPU session of measurements for profiles/<round>: GPU tests, the default
# bench line (traffic PMC + CPU baseline) with its rocprofv3 kernel stats, and
# per-kernel PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit) of the default workload.
# Stops at the first step that fails, faults or times out.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
R=${ROUND:-r2}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  local T0=$(date +%s)
  timeout -k 10 "$t" "$@" > gpurun_out/${R}_${name}.log 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - T0 )) s)"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for s in ${STEPS:-tests bench prof pmc}; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -rf ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    probe) step probe 300 python tools/gather_probe.py ${PROBE_ARGS:-} ;;
    probe_prof) step probe_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_probe_prof -o run -- \
            python3 tools/gather_probe.py --iters 20 ${PROBE_ARGS:-} ;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
            python3 bench.py --traffic off --cpu-baseline off ${BENCH_ARGS:-} ;;
    pmc) PMC_GROUPS="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum" TAG=${R}_pmc BENCH_EXTRA="${BENCH_ARGS:-}" step pmc 400 bash tools/pmc.sh ;;
  esac
done
