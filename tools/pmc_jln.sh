# PMC passes over tools/bench_jln.py (person_cl_kernel focus).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmc_jln} PMC_CMD="python3 tools/bench_jln.py --frames 32 --steps 2" PMC_GROUPS="TCC_HIT_sum TCC_MISS_sum
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum
SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU
GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc.sh
