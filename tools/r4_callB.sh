#!/bin/bash
# Round 4 GPU call B: person-kernel probe + JLN A/B (unsigned-max planes), PMC of the C5 gathers (cameras
# inner vs camera-outer rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in jwin jpf1 jpf2; do
  FVP_LIB=$PWD/ab_libs/$lib.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
    tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
    > gpurun_out/r4b_person_tests_$lib.log 2>&1 || { tail -30 gpurun_out/r4b_person_tests_$lib.log; exit 1; }
  echo "$lib person tests: $(tail -1 gpurun_out/r4b_person_tests_$lib.log)"
done
timeout -k 10 300 python3 tools/person_probe.py --iters 20 > gpurun_out/r4b_person_probe.jsonl 2>&1 || { tail -20 gpurun_out/r4b_person_probe.jsonl; exit 1; }
cat gpurun_out/r4b_person_probe.jsonl
LIBS="ab_libs/jbase.so ab_libs/jplanes_u.so ab_libs/jwin.so ab_libs/jpf1.so ab_libs/jpf2.so" REPS=2 bash tools/r4_ab_jln.sh || exit 1
for lib in pbase co1; do
  TAG=r4b_pmc_$lib PMC_CMD="python3 bench.py --workload c5 --batch 8 --child --steps 3 --warmup 1 --traffic off --cpu-baseline off" \
  PMC_GROUPS="TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  FVP_LIB=$PWD/ab_libs/$lib.so bash tools/pmc.sh > gpurun_out/r4b_pmc_$lib.txt 2>&1 || { tail -10 gpurun_out/r4b_pmc_$lib.txt; exit 1; }
  grep -A12 "voxelize_c" gpurun_out/r4b_pmc_$lib.txt | head -30
done
echo callB done
