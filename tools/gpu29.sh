set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/test_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/test_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bs128.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/bench_bs16.log 2>&1
rc=$?
tail -n1 gpurun_out/bench_bs128.log | cut -c1-160; tail -n1 gpurun_out/bench_bs16.log | cut -c1-160
exit $rc
