set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/test_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/test_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/bench_bs16.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 --graph 1 > gpurun_out/bench_bs16_graph.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --graph 1 > gpurun_out/bench_bs128_graph.log 2>&1
rc=$?
tail -1 gpurun_out/bench_bs16.log gpurun_out/bench_bs16_graph.log gpurun_out/bench_bs128_graph.log
exit $rc
