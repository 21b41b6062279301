set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/test_gpu.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --ops wgrad --iters 10 > gpurun_out/kbench_wgrad.jsonl 2>gpurun_out/kbench_wgrad.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_hip_bs128.log 2>&1
rc=$?
tail -3 gpurun_out/test_gpu.log
echo exit $rc
exit $rc
