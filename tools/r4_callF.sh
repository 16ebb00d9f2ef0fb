#!/bin/bash
# Round 4 GPU call F: person kernel occupancy caps (jmb6 / jmb7 = 6 / 7 waves per SIMD) against
# jred (the product: VALU slot reduction, div_pair on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LIBS="ab_libs/jred.so ab_libs/jmb6.so ab_libs/jmb7.so ab_libs/jmb6_pf1.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
for v in jmb6 jmb7; do
  FVP_LIB=$PWD/ab_libs/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
    > gpurun_out/r4f_${v}_tests.log 2>&1 || { tail -30 gpurun_out/r4f_${v}_tests.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/r4f_${v}_tests.log)"
done
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4f_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4f_person_probe.jsonl; exit 1; }
cat gpurun_out/r4f_person_probe.jsonl
echo callF done
