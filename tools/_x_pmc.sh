set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6_ccp; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
n=0
for p in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -f csv -d $O/p$n -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench_cond_conv.py 256 > $O/p$n.log 2>&1 || exit 1
  f=$(find $O/p$n -name '*counter_collection.csv' | head -n1)
  python3 $GRAFT_REPO_ROOT/tools/pmcstats.py "$f" conv_halo > $O/stats_p$n.txt
done
find $O -name '*.csv' -delete
