#!/bin/bash
# Round 4 GPU call J: kernel trace of the JLN line (where the op's time beyond the person kernel
# goes), and the C2 gather's TD / TA / L2 / SQ counters at the shipped kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_jln -o run -- \
  python3 tools/bench_jln.py --frames 32 --steps 10 > $OUT/ks_jln.log 2>&1 || { tail -5 $OUT/ks_jln.log; exit 1; }
python3 tools/kstats.py $OUT/ks_jln
TAG=r4j/pmc_c2 BENCH_EXTRA="--workload c2" PMC_GROUPS="TCC_HIT_sum TCC_MISS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
  bash tools/pmc.sh > $OUT/pmc_c2.txt 2>&1 || { tail -5 $OUT/pmc_c2.txt; exit 1; }
grep -A 20 "voxelize_kernel" $OUT/pmc_c2.txt | head -22
FVP_LIB=$PWD/ab_libs/jrp2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "person or jln or e2e or individual" \
  > $OUT/jrp2_tests.log 2>&1 || { tail -30 $OUT/jrp2_tests.log; exit 1; }
echo "jrp2 tests: $(tail -1 $OUT/jrp2_tests.log)"
LIBS="ab_libs/jdxy.so ab_libs/jrp2.so" REPS=3 bash tools/r4_ab_jln.sh || exit 1
echo callJ done
