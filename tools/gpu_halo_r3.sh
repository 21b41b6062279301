set -o pipefail
mkdir -p gpurun_out/halo
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "conv or halo or graph_step_bitwise" --timeout 120 --timeout-method thread > gpurun_out/halo/tests.txt 2>&1 || { tail -30 gpurun_out/halo/tests.txt; exit 1; }
tail -3 gpurun_out/halo/tests.txt
timeout -k 10 200 python -u tools/kbench_conv_epi_r3.py 256 > gpurun_out/halo/kbench.txt 2>&1 && cat gpurun_out/halo/kbench.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/halo/b128.txt 2>&1 && tail -1 gpurun_out/halo/b128.txt
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --global_batch 16 > gpurun_out/halo/b16.txt 2>&1 && tail -1 gpurun_out/halo/b16.txt
