set -o pipefail
cd /root/repo && export PYTHONPATH=/root/repo
mkdir -p gpurun_out
for gm in 1 2 4 8 16; do
  echo "gm=$gm"
  timeout -k 10 200 python tools/kbench_gemm.py --vers 3 --gm $gm --rounds 2 --iters 10 --only "${SHAPE:-film fwd}" 2> gpurun_out/kg_gm.err || exit $?
done
