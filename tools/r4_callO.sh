#!/bin/bash
# Round 4 GPU call O: tile kernel with the xz maxima accumulated in LDS and sent as 64-B runs
# every 8 / 16 x steps (jtl8 / jtl16) against the row kernel (jxyd) and the register batch (jtile8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4o
FVP_LIB=$PWD/ab_libs/jtl8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py tests/test_backbone.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual or channels" \
  > gpurun_out/r4o/jtl8_tests.log 2>&1 || { tail -30 gpurun_out/r4o/jtl8_tests.log; exit 1; }
echo "jtl8 tests: $(tail -1 gpurun_out/r4o/jtl8_tests.log)"
LIBS="ab_libs/jxyd.so ab_libs/jtile8.so ab_libs/jtl8.so ab_libs/jtl16.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
echo callO done
