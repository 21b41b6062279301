# bs16 (the 8-GPU per-GPU share): FiLM weight gradient on the split-K MFMA
# kernel (auto at <= 32 frames) vs the hipBLASLt split-K slabs (blas).
set -o pipefail
O=gpurun_out/fw16; mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do for v in auto blas; do
  D3D_FILM_WGRAD=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --global_batch 16 > $O/b16_$v.json 2>$O/b16_$v.err || exit $?
  echo "b16 film_wgrad=$v $(show $O/b16_$v.json)"
done; done
