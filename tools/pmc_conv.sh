set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcconv; mkdir -p $O
P="python3 $R/tools/conv_layer_probe.py --iters 10"
timeout -k 10 120 $P > $O/probe.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/p1 -o run -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE -d $O/p2 -o run -- $P > /dev/null
echo done
