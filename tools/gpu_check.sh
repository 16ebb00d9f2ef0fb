#!/bin/bash
# One GPU session: parity tests, smoke, short bench (+ optional rocprofv3 stats).
# Stops at the first step that faults, aborts or times out (rc 124/134/137/139 or >128).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] && [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in ${STEPS:-pytest smoke bench}; do
  case $step in
    pytest) run pytest 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ;;
    pytestall) run pytestall 400 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ;;
    smoke) run smoke 150 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --traffic off --cpu-seconds 5} ;;
    prof) run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --traffic off --cpu-baseline off ;;
    taprobe) run taprobe 400 python tools/ta_probe.py ;;
  esac
done
