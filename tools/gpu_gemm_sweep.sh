set -o pipefail
mkdir -p gpurun_out/gemm2
export PYTHONPATH=.
timeout -k 10 200 python tools/kbench_gemm.py > gpurun_out/gemm2/gm4.txt 2>&1 || exit $?
D3D_GEMM_GM=64 timeout -k 10 200 python tools/kbench_gemm.py --only film > gpurun_out/gemm2/gm64.txt 2>&1 || exit $?
D3D_GEMM_GM=8 timeout -k 10 200 python tools/kbench_gemm.py --only film > gpurun_out/gemm2/gm8.txt 2>&1 || exit $?
D3D_GEMM_GRID=100000 timeout -k 10 200 python tools/kbench_gemm.py --only film > gpurun_out/gemm2/nonpersist.txt 2>&1 || exit $?
