# GN backward reduce tail (SoA LDS + lane-team group sums): GN GPU tests, interleaved A/B against
# libd3d_hip_old.so at bs16 and bs128, and the kernel's LDS conflict share per build (bs16 step, --pmc)
set -o pipefail
O=/root/repo/gpurun_out/abg
mkdir -p $O
OLD=/root/repo/distributed_3d_diffusion_pytorch_amd/ops/libd3d_hip_old.so
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "group_norm or gn or film or graph_step_bitwise" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {  # name, lib, args
  local name=$1; shift
  local lib=$1; shift
  D3D_LIB_PATH=$lib timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run b16_old_$r $OLD --global_batch 16 --steps 40 --warmup 8 || exit 1
  run b16_new_$r "" --global_batch 16 --steps 40 --warmup 8 || exit 1
done
for r in 1 2; do
  run b128_old_$r $OLD --steps 15 --warmup 4 || exit 1
  run b128_new_$r "" --steps 15 --warmup 4 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  lib=""; [ $v = old ] && lib=$OLD
  D3D_LIB_PATH=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/pmc_$v -o run -- python3 /root/repo/bench.py --global_batch 16 --steps 2 --warmup 1 > $O/pmc_$v.log 2>&1 || { tail -5 $O/pmc_$v.log; exit 1; }
  python3 /root/repo/tools/pmc_step_table.py $O/pmc_$v $O/pmc_$v $O/pmc_$v > $O/pmc_$v.txt 2>&1
  echo "== $v"; grep gn_ $O/pmc_$v.txt
done
find $O -name '*.csv' -delete
