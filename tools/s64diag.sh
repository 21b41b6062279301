set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s64a; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u tools/kbench_s64.py --dgrad > $O/kb.txt 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -f csv -d $O/p1 -o run -- python3 $R/tools/kbench_s64.py --shapes 0,1 --cfgs 0 --dgrad --iters 5 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM --kernel-trace -f csv -d $O/p2 -o run -- python3 $R/tools/kbench_s64.py --shapes 0,1 --cfgs 0 --dgrad --iters 5 > $O/p2.log 2>&1
echo done
