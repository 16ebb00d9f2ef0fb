#!/bin/bash
# Round 4 GPU call C: the -m gpu suite at HEAD, the person-kernel replay probe, and the
# JLN A/B (jbase = the person kernel before the unsigned-max planes / window walk,
# jcur = HEAD, jpf1 / jpf2 = HEAD with the grid prefetch ring, jyg2 / jyg4 = 2 / 4 rows
# per block, jpipe = two-stage camera pipeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r4c WORKLOADS="c2:256" bash tools/r3_check.sh || exit 1
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4c_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4c_person_probe.jsonl; exit 1; }
cat gpurun_out/r4c_person_probe.jsonl
LIBS="ab_libs/jbase.so ab_libs/jcur.so ab_libs/jpf1.so ab_libs/jpf2.so ab_libs/jyg2.so ab_libs/jyg4.so ab_libs/jpipe.so ab_libs/jpipe_pf1.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
FVP_LIB=$PWD/ab_libs/jpipe.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
  > gpurun_out/r4c_jpipe_tests.log 2>&1 || { tail -30 gpurun_out/r4c_jpipe_tests.log; exit 1; }
echo "jpipe tests: $(tail -1 gpurun_out/r4c_jpipe_tests.log)"
LIBS="ab_libs/vbase.so ab_libs/vpipe.so ab_libs/vpipe8.so ab_libs/vpipe5.so" WL="c2:256" REPS=2 TAG=vpipe bash tools/r4_ab_c5.sh || exit 1
echo callC done
