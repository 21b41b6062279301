# PMC counter passes over the halo (direct) 3x3 conv -- the top kernel of the
# bs128 step -- on the 64x64-level shapes, forward and input gradient, against
# the implicit-GEMM w8 kernel on the same shape (one counter group per run).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/pmc_halo
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM"
for impl in halo w8w; do
 for shp in "--h 64 --ci 128 --co 128" "--h 64 --ci 384 --co 128" "--h 64 --ci 128 --co 128 --dgrad"; do
  tag=$impl$(echo $shp | tr -d ' -')
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/$tag.p1 -o run --output-format csv -- python3 /root/repo/tools/conv_one.py --impl $impl $shp --iters 5 > $O/$tag.p1.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/$tag.p2 -o run --output-format csv -- python3 /root/repo/tools/conv_one.py --impl $impl $shp --iters 5 > $O/$tag.p2.log 2>&1 || exit $?
  for p in p1 p2; do f=$(find $O/$tag.$p -name '*counter_collection.csv' | head -n1); python3 /root/repo/tools/pmcstats.py $f conv_ > $O/$tag.$p.txt; done
  rm -rf $O/$tag.p1 $O/$tag.p2
 done
done
for impl in halo w8w; do for shp in "--h 64 --ci 128 --co 128" "--h 64 --ci 384 --co 128" "--h 64 --ci 128 --co 128 --dgrad"; do
  timeout -k 10 60 python3 /root/repo/tools/conv_one.py --impl $impl $shp || exit $?; done; done > $O/timing.txt
cat $O/timing.txt
