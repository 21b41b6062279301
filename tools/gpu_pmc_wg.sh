# PMC counter passes over the grouped weight-gradient kernel (tools/kbench_wgrad_group.py
# L0 / L1 3x3 batches at bs128 and bs16 shapes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/pmcwg
mkdir -p $O
(cd /root/repo && timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "group_norm or cat_gn or gn_film or full_model" > $O/pytest.log 2>&1) || { tail -20 $O/pytest.log; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"
P3="FETCH_SIZE SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for ex in 128 16; do
  for b in "L0 3x3" "L1 3x3"; do
    tag=e${ex}_$(echo $b | tr -d ' ')
    for p in 1 2 3; do
      eval C=\$P$p
      timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/$tag.p$p -o run --output-format csv -- python3 /root/repo/tools/kbench_wgrad_group.py --examples $ex --only "$b" --skip_old --iters 3 > $O/$tag.p$p.log 2>&1 || exit $?
      f=$(find $O/$tag.p$p -name '*counter_collection.csv' | head -n1); python3 /root/repo/tools/pmcstats.py $f wgrad_grp > $O/$tag.p$p.txt
    done
  done
done
timeout -k 10 120 python3 /root/repo/tools/kbench_wgrad_group.py --examples 128 --skip_old > $O/kb128.jsonl
true
