set -o pipefail
mkdir -p gpurun_out/r6_gm
for gm in 2 4 8 16 64; do
  timeout -k 10 300 python3 tools/kbench_gemm.py --only "film fwd P1" --rounds 2 --iters 10 --gm $gm > gpurun_out/r6_gm/gm$gm.txt 2>&1 || exit 1
done
