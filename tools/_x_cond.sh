set -o pipefail
mkdir -p gpurun_out/r6_ocl
timeout -k 10 200 python3 tools/kbench_cond_conv.py 256 > gpurun_out/r6_ocl/k256.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/kbench_cond_conv.py 32 > gpurun_out/r6_ocl/k32.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "cond or ray or full_model or conv3x3 or graph_train_step or bitwise" > gpurun_out/r6_ocl/tests.log 2>&1 || { tail -30 gpurun_out/r6_ocl/tests.log; exit 1; }
tail -1 gpurun_out/r6_ocl/tests.log
