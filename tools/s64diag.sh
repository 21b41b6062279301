# PMC passes over the small-level conv kbench (usage: bash tools/s64diag.sh <out> [kbench args...])
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --kernel-trace -f csv -d $O/p1 -o run -- python3 $R/tools/kbench_s64.py "$@" > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES --kernel-trace -f csv -d $O/p2 -o run -- python3 $R/tools/kbench_s64.py "$@" > $O/p2.log 2>&1
echo done
