# weight-gradient job batch size inside the graph (D3D_WGRAD_DEFER_BATCH) at bs16 / bs32, two interleaved rounds
set -o pipefail
cd /root/repo
O=gpurun_out/wdb
mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for v in 32 64 1000; do
    D3D_WGRAD_DEFER_BATCH=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$v.json 2> $O/b16_$v.err || exit $?
    echo "b16 batch=$v $(show $O/b16_$v.json)"
  done
done
for r in 1 2; do
  for v in 8 64; do
    D3D_WGRAD_DEFER_BATCH=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --global_batch 32 > $O/b32_$v.json 2> $O/b32_$v.err || exit $?
    echo "b32 batch=$v $(show $O/b32_$v.json)"
  done
done
