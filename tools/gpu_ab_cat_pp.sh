# Virtual-concat NIN skip forward on the hand-written ping-pong GEMM (D3D_CAT_PP=1)
# vs two accumulating hipBLASLt GEMMs (0), interleaved, bs128 / bs32 / bs16.
set -o pipefail
O=gpurun_out/catpp; mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do for v in 1 0; do
  D3D_CAT_PP=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_$v.json 2>$O/b128_$v.err || exit $?
  echo "b128 cat_pp=$v $(show $O/b128_$v.json)"
  D3D_CAT_PP=$v timeout -k 10 300 python bench.py --steps 30 --warmup 4 --global_batch 16 > $O/b16_$v.json 2>$O/b16_$v.err || exit $?
  echo "b16  cat_pp=$v $(show $O/b16_$v.json)"
done; done
