set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "conv3x3" > $O/test_w8.log 2>&1
rc=$?; tail -n 4 $O/test_w8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops conv,dgrad --iters 10 --batch 64 > $O/kbench_w8.jsonl 2>$O/kbench_w8.err || exit $?
grep -v wgrad $O/kbench_w8.jsonl
