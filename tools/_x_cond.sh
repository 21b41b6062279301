set -o pipefail
mkdir -p gpurun_out/r6_cc
timeout -k 10 200 python3 tools/kbench_cond_conv.py 256 > gpurun_out/r6_cc/base.txt 2>&1 || exit 1
D3D_LIB_PATH=ablib/halodirect/libd3d_hip.so timeout -k 10 200 python3 tools/kbench_cond_conv.py 256 > gpurun_out/r6_cc/direct.txt 2>&1 || exit 1
