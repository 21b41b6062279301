# PMC passes over the conditioning-conv kbench (usage: bash tools/cc_pmc.sh <out> [frames])
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; N=${2:-256}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -f csv -d $O/p1 -o run -- python3 $R/tools/kbench_cond_conv.py $N > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum --kernel-trace -f csv -d $O/p2 -o run -- python3 $R/tools/kbench_cond_conv.py $N > $O/p2.log 2>&1
echo done
