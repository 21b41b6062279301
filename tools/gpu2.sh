set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -x -q -m gpu > gpurun_out/test_ops_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/test_ops_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --global_batch 16 > gpurun_out/bench_hip_bs16.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --profile gpurun_out/prof_hip_bs128.txt > gpurun_out/bench_hip_bs128.log 2>&1
echo exit $?
