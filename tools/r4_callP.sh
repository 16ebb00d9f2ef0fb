#!/bin/bash
# Round 4 GPU call P: what the person kernel's xz atomics cost -- PMC over the replay probe
# (FULL vs NO_XZ_ATOMICS etc. are separate kernel instantiations, so one pass per group covers
# every mode), and the counter list of this gfx950 for the atomic / write counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out/r4p
timeout -k 10 120 rocprofv3 -L > gpurun_out/r4p/counters.txt 2>&1 || true
grep -io "TC[CP]_[A-Z0-9_]*ATOM[A-Z0-9_]*\|TCC_EA0_WR[A-Z0-9_]*\|SQ_INSTS_VMEM_WR\|SQ_INSTS_FLAT" gpurun_out/r4p/counters.txt | sort -u | head -40
TAG=r4p/pmc PMC_CMD="python3 tools/person_probe.py --iters 3" PMC_GROUPS="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS
TCC_HIT_sum TCC_MISS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
GRBM_GUI_ACTIVE GRBM_COUNT
WRITE_SIZE" bash tools/pmc.sh > gpurun_out/r4p/pmc.txt 2>&1 || { tail -5 gpurun_out/r4p/pmc.txt; exit 1; }
grep -A 18 "person_cl_kernel<4, false, false, 0>\|person_cl_kernel<4, false, false, 5>\|person_cl_kernel<4, false, false, 1>" gpurun_out/r4p/pmc.txt | head -80
echo callP done
