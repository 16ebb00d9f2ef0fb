#!/bin/bash
# Round 4 GPU call H: staggered x walk in the person kernel (jstag) against the product (jdxy):
# parity + JLN A/B; then the C4 / C5 bench lines with the traffic PMC (tools/r4_c45.sh lines).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
FVP_LIB=$PWD/ab_libs/jstag.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
  > gpurun_out/r4h_jstag_tests.log 2>&1 || { tail -30 gpurun_out/r4h_jstag_tests.log; exit 1; }
echo "jstag tests: $(tail -1 gpurun_out/r4h_jstag_tests.log)"
LIBS="ab_libs/jdxy.so ab_libs/jstag.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
SKIP_STATS=1 bash tools/r4_c45.sh || exit 1
echo callH done
