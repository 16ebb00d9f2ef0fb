#!/bin/bash
# Round 4 GPU call L: the cleaned person kernel (jxyd) against jdxy: parity, probe, JLN A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
  > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r4l_tests.log)"
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4l_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4l_person_probe.jsonl; exit 1; }
cat gpurun_out/r4l_person_probe.jsonl
LIBS="ab_libs/jdxy.so ab_libs/jxyd.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
echo callL done
