set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests/test_ops_gpu.py -x -q -k "conv or linear or film or model or sink or graph" > gpurun_out/test_conv.log 2>&1
rc=$?; tail -3 gpurun_out/test_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops wgrad --iters 10 --batch 64 > gpurun_out/kbench_wgrad_bufl.jsonl 2>gpurun_out/kbench.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bs128.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/bench_bs16.log 2>&1
rc=$?
tail -n1 gpurun_out/bench_bs128.log | cut -c1-160; tail -n1 gpurun_out/bench_bs16.log | cut -c1-160
exit $rc
