#!/bin/bash
# 8-entry pair layout kernel: fp16 parity + digest tests on the in-tree build, then a same-box
# A/B (vec8 vs rows) on C5/C4 bench lines with kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/r4R; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LIBS="ab_libs/p8.so ab_libs/prows.so" WL="c5:8 c5:32 c4:32" REPS=2 KSTATS=c5:8 TAG=r4R bash tools/r4_ab_c5.sh
