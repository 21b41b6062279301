# Dense GEMM activation-stream cache policy (ablib/<variant> built with -DD3D_GEMM_B_CPOL=<n>) vs the
# in-tree library: FiLM kernels in isolation, then the step with the FiLM forward on gemm_fw_k.
set -o pipefail
V=${1:?variant}; O=gpurun_out/${2:-r6_cpol}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/kbench_gemm.py --only "film" --rounds 2 --iters 10 > $O/k_base_$r.txt 2>&1 || exit 1
  D3D_LIB_PATH=ablib/$V/libd3d_hip.so timeout -k 10 300 python3 -u tools/kbench_gemm.py --only "film" --rounds 2 --iters 10 > $O/k_${V}_$r.txt 2>&1 || exit 1
done
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  D3D_FILM_BLAS=0 timeout -k 10 300 python3 -u bench.py --global_batch 128 --steps 15 --warmup 4 > $O/b_base_$r.json 2>/dev/null || exit 1
  echo "bench FILM_BLAS=0 base r$r $(v $O/b_base_$r.json)"
  D3D_FILM_BLAS=0 D3D_LIB_PATH=ablib/$V/libd3d_hip.so timeout -k 10 300 python3 -u bench.py --global_batch 128 --steps 15 --warmup 4 > $O/b_${V}_$r.json 2>/dev/null || exit 1
  echo "bench FILM_BLAS=0 $V r$r $(v $O/b_${V}_$r.json)"
  timeout -k 10 300 python3 -u bench.py --global_batch 128 --steps 15 --warmup 4 > $O/b_blas_$r.json 2>/dev/null || exit 1
  echo "bench default (blas) r$r $(v $O/b_blas_$r.json)"
done
