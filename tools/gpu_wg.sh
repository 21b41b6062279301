set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "wgrad_w8 or conv3x3" > $O/test_wg.log 2>&1
rc=$?; tail -n 4 $O/test_wg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops wgrad --iters 10 --batch 64 > $O/kbench_wg.jsonl 2>$O/kbench_wg.err || exit $?
cat $O/kbench_wg.jsonl
