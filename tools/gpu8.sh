set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "conv or linear or sink" > gpurun_out/test_ops_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/test_ops_gpu.log
tail -2 gpurun_out/test_ops_gpu.log
timeout -k 10 600 python tools/kbench.py --ops wgrad --iters 10 > gpurun_out/kbench_wgrad.jsonl 2>/dev/null
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --profile gpurun_out/prof_hip_bs128.txt > gpurun_out/bench_hip_bs128.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/bench_hip_bs16.log 2>&1
echo exit $?
