# PMC passes: level-0 halo conv fwd / dgrad (tools/conv_one.py) next to the halo weight gradient
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/pmc_conv4
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"
for shp in "--h 64 --ci 128 --co 128" "--h 64 --ci 128 --co 128 --dgrad" "WG"; do
  tag=$(echo $shp | tr -d ' -')
  for p in 1 2; do
    eval C=\$P$p
    if [ "$shp" = WG ]; then
      cmd="python3 /root/repo/tools/kbench_wgrad_group.py --examples 128 --only L0_3x3 --skip_old --iters 3"
    else
      cmd="python3 /root/repo/tools/conv_one.py --impl halo --n 256 $shp --iters 5"
    fi
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/$tag.p$p -o run --output-format csv -- $cmd > $O/$tag.p$p.log 2>&1 || exit $?
    f=$(find $O/$tag.p$p -name '*counter_collection.csv' | head -n1); python3 /root/repo/tools/pmcstats.py $f "" > $O/$tag.p$p.txt
    rm -rf $O/$tag.p$p
  done
done
cat $O/*.txt
