set -o pipefail
cd /root/repo
for impl in reg bufl reg bufl; do
  D3D_WGRAD_IMPL=$impl timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$impl.log 2>&1 || exit 1
  echo "$impl $(tail -n1 gpurun_out/ab_$impl.log | cut -c90-130)"
done
for impl in reg bufl; do
  D3D_WGRAD_IMPL=$impl timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/ab16_$impl.log 2>&1 || exit 1
  echo "bs16 $impl $(tail -n1 gpurun_out/ab16_$impl.log | cut -c90-130)"
done
