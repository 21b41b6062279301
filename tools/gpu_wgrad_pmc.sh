# PMC pass over the TN weight-gradient GEMM (and hipBLASLt) at one FiLM shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/${TAG:-wpmc}
mkdir -p $O
export PYTHONPATH=/root/repo
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 /root/repo/tools/kbench_wgrad_tn.py --only ${ROWS:-1048576} --iters 3 > $O/p1.log 2>&1 || exit $?
python3 /root/repo/tools/pmc_summary.py $O/p1 > $O/summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 /root/repo/tools/kbench_wgrad_tn.py --only ${ROWS:-1048576} --iters 3 > $O/p2.log 2>&1 || exit $?
python3 /root/repo/tools/pmc_summary.py $O/p2 >> $O/summary.txt
cat $O/summary.txt
