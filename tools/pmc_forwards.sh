#!/bin/bash
# MFMA evidence of the shipped CNN forwards: for each net, a
# kernel trace of 8 forwards (per-dispatch durations, tools/cnn_trace.py parse) and
# one PMC pass (MFMA busy, SQ busy, GPU-active cycles, MFMA ops issued) over the
# same forwards (tools/cnn_trace.py pmc: per dispatch of the last forward and the
# forward's totals).  Output under gpurun_out/${OUT:-pmcfwd}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
O=gpurun_out/${OUT:-pmcfwd}; mkdir -p $O
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE"
# (third field: the fewest dispatches a forward has -- trace groups below it are setup work)
for spec in "p2p 240 10" "centernet 8 10" "c2c 80 1" "backbone 40 10"; do
  set -- $spec; net=$1; n=$2; per=$3
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$net -o run -- python3 tools/cnn_trace.py run --net $net --images $n > $O/tr_$net.log 2>&1 || { echo "trace $net failed"; tail -20 $O/tr_$net.log; exit 1; }
  python3 tools/cnn_trace.py parse $O/tr_$net --min-dispatches $per > $O/trace_$net.json || exit 1
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$net -o run -- python3 tools/cnn_trace.py run --net $net --images $n --iters 3 > $O/pmc_$net.log 2>&1 || { echo "pmc $net failed"; tail -20 $O/pmc_$net.log; exit 1; }
  per=$(python3 -c "import json; print(json.load(open('$O/trace_$net.json'))['dispatches'])")
  python3 tools/cnn_trace.py pmc $O/pmc_$net --per-forward $per > $O/pmc_$net.jsonl || exit 1
  echo "$net: $(python3 -c "import json; t=json.load(open('$O/trace_$net.json')); print('busy_us', t['last_busy_us'], 'dispatches', t['dispatches'])") $(tail -1 $O/pmc_$net.jsonl)"
  rm -rf $O/tr_$net $O/pmc_$net
done
