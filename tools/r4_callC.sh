#!/bin/bash
# Round 4 GPU call C: the -m gpu suite at HEAD, the person-kernel replay probe, and the
# JLN A/B (jbase = the person kernel before the unsigned-max planes / window walk,
# jcur = HEAD, jpf1 / jpf2 = HEAD with the grid prefetch ring).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r4c WORKLOADS="c2:256" bash tools/r3_check.sh || exit 1
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4c_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4c_person_probe.jsonl; exit 1; }
cat gpurun_out/r4c_person_probe.jsonl
LIBS="ab_libs/jbase.so ab_libs/jcur.so ab_libs/jpf1.so ab_libs/jpf2.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1

LIBS="ab_libs/pbase.so ab_libs/dp.so" WL="c5:8 c5:32" REPS=2 TAG=dp bash tools/r4_ab_c5.sh || exit 1
FVP_LIB=$PWD/ab_libs/dp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_dp_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c_dp_tests.log; exit 1; }
echo "dp tests: $(tail -1 gpurun_out/r4c_dp_tests.log)"
echo callC2 done
