#!/bin/bash
# PMC passes over one conv layer (tools/conv_layer_probe.py; PROBE_ARGS picks
# the layer, TAG the output directory), summarised on the box by pmc_db.py.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcconv${TAG:+_$TAG}; mkdir -p $O
P="python3 $R/tools/conv_layer_probe.py --iters 10 ${PROBE_ARGS:-}"
timeout -k 10 120 $P > $O/probe.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/p1 -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d $O/p2 -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum -d $O/p4 -o run -- $P > /dev/null
for d in p1 p2 p3 p4; do python3 $R/tools/pmc_db.py --match conv $O/$d > $O/$d.txt; rm -rf $O/$d; done
echo done
