#!/bin/bash
# Round 4 GPU call S: the x-part person kernel (jxp: xz / xy maxima in LDS for the block's
# x-planes, yz atomics per row) against the row kernel (jxyd): parity + JLN A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4s
FVP_LIB=$PWD/ab_libs/jxp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py tests/test_backbone.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual or channels" \
  > gpurun_out/r4s/jxp_tests.log 2>&1 || { tail -30 gpurun_out/r4s/jxp_tests.log; exit 1; }
echo "jxp tests: $(tail -1 gpurun_out/r4s/jxp_tests.log)"
LIBS="ab_libs/jxyd.so ab_libs/jxp.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
echo callS done
