set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_ops_gpu.py -x -q -m gpu > gpurun_out/test_ops_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/test_ops_gpu.log
tail -3 gpurun_out/test_ops_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_hip_bs128.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --global_batch 16 --profile gpurun_out/prof_hip_bs16.txt > gpurun_out/bench_hip_bs16.log 2>&1 && \
timeout -k 10 600 python bench.py --mode sample --warmup 3 > gpurun_out/bench_sample.log 2>&1
echo exit $?
