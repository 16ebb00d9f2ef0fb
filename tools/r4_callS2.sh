#!/bin/bash
# The 8-entry pair layout for single-frame entries too (v8one) against it for frame groups only
# (v8multi): fp16 parity tests on the in-tree (v8one) build, C5 B=1 / B=5 bench lines, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; O=gpurun_out/r4S2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_digests.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LIBS="ab_libs/v8one.so ab_libs/v8multi.so" WL="c5:1 c5:5 c5:8" REPS=2 KSTATS=c5:1 TAG=r4S2 bash tools/r4_ab_c5.sh
