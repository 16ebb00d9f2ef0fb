#!/bin/bash
# (Ran on a temporary build with person_cl_kernel<..., RW=4> and its FVP_PERSON_ROWS knob; both were removed.)
# Person planes: 4-row x 16-z blocks (default) vs one-row 64-z blocks (FVP_PERSON_ROWS=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-person}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
FVP_PERSON_ROWS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "jln or person or planes or JLN" > gpurun_out/${T}_tests_rows1.log 2>&1 || { tail -40 gpurun_out/${T}_tests_rows1.log; exit 1; }
tail -1 gpurun_out/${T}_tests_rows1.log
for rep in 1 2; do
  for r in 1 4; do
    FVP_PERSON_ROWS=$r timeout -k 10 300 python3 tools/bench_jln.py --frames 32 > gpurun_out/${T}_jln_r${r}_$rep.log 2>&1 || { tail -20 gpurun_out/${T}_jln_r${r}_$rep.log; exit 1; }
    echo "rows$r rep$rep $(grep '^{' gpurun_out/${T}_jln_r${r}_$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['us_per_proposal'], d.get('per_frame_us_per_proposal', d.get('per_frame_calls_us_per_proposal')))")"
  done
done
