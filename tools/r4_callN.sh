#!/bin/bash
# Round 4 GPU call N: the 4 x 4-tile person kernel (jtile) against the row kernel (jxyd):
# parity on the JLN / person tests, the replay probe (both kernels), JLN A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4n
FVP_LIB=$PWD/ab_libs/jtile8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py tests/test_backbone.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual or channels" \
  > gpurun_out/r4n/jtile_tests.log 2>&1 || { tail -30 gpurun_out/r4n/jtile_tests.log; exit 1; }
echo "jtile tests: $(tail -1 gpurun_out/r4n/jtile_tests.log)"
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4n/person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4n/person_probe.jsonl; exit 1; }
cat gpurun_out/r4n/person_probe.jsonl
LIBS="ab_libs/jxyd.so ab_libs/jtile8.so ab_libs/jtile4.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
echo callN done
