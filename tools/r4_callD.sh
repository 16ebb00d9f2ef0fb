#!/bin/bash
# Round 4 GPU call D: same-box A/B of the C5 gather with div_pair (dp) and of the C2 / C4
# gathers with the two-stage camera pipeline (vpipe), each with its parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LIBS="ab_libs/vbase.so ab_libs/vpipe.so ab_libs/vpipe8.so ab_libs/vpipe5.so" WL="c2:256 c4:64" REPS=2 TAG=vpipe bash tools/r4_ab_c5.sh || exit 1
LIBS="ab_libs/pbase.so ab_libs/dp.so" WL="c5:8 c5:32" REPS=2 TAG=dp bash tools/r4_ab_c5.sh || exit 1
for v in vpipe dp; do
  FVP_LIB=$PWD/ab_libs/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_${v}_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4d_${v}_tests.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r4d_${v}_tests.log)"
done
echo callD done
