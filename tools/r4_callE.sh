#!/bin/bash
# Round 4 GPU call E: person kernel with the VALU slot reduction for the xy plane (jred; jred_pf1 with
# the grid prefetch ring) against jcur, its parity tests, the replay probe; then the C5 div_pair A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in jred jred_pf1; do
  FVP_LIB=$PWD/ab_libs/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
    > gpurun_out/r4e_${v}_tests.log 2>&1 || { tail -30 gpurun_out/r4e_${v}_tests.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r4e_${v}_tests.log)"
done
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4e_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4e_person_probe.jsonl; exit 1; }
cat gpurun_out/r4e_person_probe.jsonl
LIBS="ab_libs/jcur.so ab_libs/jred.so ab_libs/jred_pf1.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
LIBS="ab_libs/pbase.so ab_libs/dp.so" WL="c5:8 c5:32" REPS=2 TAG=dp bash tools/r4_ab_c5.sh || exit 1
FVP_LIB=$PWD/ab_libs/dp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_dp_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4e_dp_tests.log; exit 1; }
echo "dp tests: $(tail -1 gpurun_out/r4e_dp_tests.log)"
echo callE done
