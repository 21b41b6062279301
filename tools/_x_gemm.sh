set -o pipefail
mkdir -p gpurun_out/r6_x
for v in base xskipb xzerob; do
  if [ $v = base ]; then unset D3D_LIB_PATH; else export D3D_LIB_PATH=ablib/$v/libd3d_hip.so; fi
  timeout -k 10 200 python3 tools/kbench_gemm.py --only "film fwd P1" --rounds 2 --iters 10 > gpurun_out/r6_x/$v.txt 2>&1 || exit 1
done
unset D3D_LIB_PATH
timeout -k 10 300 python3 bench.py --global_batch 16 --graph 0 --steps 3 --warmup 3 --profile gpurun_out/r6_x/glue16.txt --profile_stack 8 > gpurun_out/r6_x/b16p.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --global_batch 128 --steps 2 --warmup 2 --profile gpurun_out/r6_x/glue128.txt --profile_stack 8 > gpurun_out/r6_x/b128p.log 2>&1 || exit 1
