#!/bin/bash
# Round 4 GPU call A: the -m gpu suite, parity of the A/B variants on the C5 / fp16 tests, the person-kernel
# replay probe, JLN and C5 A/B lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r4a WORKLOADS="c2:256 c5:8" bash tools/r3_check.sh || exit 1
for v in pvec_mdiv co1; do
  FVP_LIB=$PWD/ab_libs/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_digests.py tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "c5 or fp16 or f16 or nonfinite" \
    > gpurun_out/r4a_${v}_tests.log 2>&1 || { tail -30 gpurun_out/r4a_${v}_tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r4a_${v}_tests.log)"
done
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4a_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4a_person_probe.jsonl; exit 1; }
cat gpurun_out/r4a_person_probe.jsonl
LIBS="ab_libs/jbase.so ab_libs/jnt.so ab_libs/jxs2.so ab_libs/jnt_xs2.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
LIBS="ab_libs/pbase.so ab_libs/co1.so ab_libs/co2.so ab_libs/co1lb.so ab_libs/pvec.so ab_libs/mdiv.so ab_libs/gnt.so" \
  WL="c5:8" REPS=1 bash tools/r4_ab_c5.sh || exit 1
LIBS="ab_libs/pbase.so ab_libs/co1.so" WL="c5:32" REPS=1 KSTATS="c5:8" bash tools/r4_ab_c5.sh || exit 1
echo callA done
