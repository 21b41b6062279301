set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "cond_conv or wgrad or conv3x3" > $O/test_wgt.log 2>&1
rc=$?; tail -n 3 $O/test_wgt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops wgrad --iters 10 --batch 16 > $O/kbw16.jsonl 2>/dev/null || exit $?
timeout -k 10 600 python tools/kbench.py --ops wgrad --iters 10 --batch 64 > $O/kbw64.jsonl 2>/dev/null || exit $?
grep -h "w8\|bufl" $O/kbw16.jsonl $O/kbw64.jsonl | cut -c1-150
