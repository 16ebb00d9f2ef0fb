#!/bin/bash
# Round 4: HBM-roofline capture of the C4 / C5 kernels that ship:
# bench lines with the FETCH_SIZE / WRITE_SIZE traffic, rocprofv3 kernel stats, and
# per-kernel PMC passes (FETCH / WRITE / TCC hit-miss / TD / TA / SQ).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
OUT=gpurun_out/r4_c45; mkdir -p $OUT
line() {  # tag args...
  local tag=$1; shift
  timeout -k 10 ${TMO:-420} python3 bench.py "$@" --steps 10 --warmup 2 --traffic auto --cpu-baseline ${CPU:-on} \
    > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; exit 1; }
  echo "$tag: $(tail -1 $OUT/bench_$tag.json | cut -c1-160)"
}
stats() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$tag -o run -- \
    python3 bench.py "$@" --steps 10 --warmup 2 --traffic off --cpu-baseline off > $OUT/ks_$tag.log 2>&1 \
    || { tail -5 $OUT/ks_$tag.log; exit 1; }
  echo "stats $tag ok"
}
pmc() {  # tag args...
  local tag=$1; shift
  TAG=r4_c45/pmc_$tag BENCH_EXTRA="$*" PMC_GROUPS="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
    bash tools/pmc.sh > $OUT/pmc_$tag.txt 2>&1 || { tail -5 $OUT/pmc_$tag.txt; exit 1; }
  echo "pmc $tag ok"
}
[ -n "${SKIP_LINES:-}" ] || {
  TMO=600 line c5_b8 --workload c5 --batch 8
  CPU=off line c5_b32 --workload c5 --batch 32
  line c4_b64 --workload c4 --batch 64
  CPU=off line c4_b32 --workload c4 --batch 32
}
[ -n "${SKIP_STATS:-}" ] && { echo done; exit 0; }
stats c5_b8 --workload c5 --batch 8
stats c4_b64 --workload c4 --batch 64
pmc c5_b8 --workload c5 --batch 8
pmc c4_b64 --workload c4 --batch 64
echo done
