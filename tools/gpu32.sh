set -o pipefail
cd /root/repo
D3D_CONV_IMPL=bufl1 timeout -k 10 900 python -m pytest tests/test_ops_gpu.py -x -q -k "conv" > gpurun_out/test_conv.log 2>&1
rc=$?; tail -2 gpurun_out/test_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops conv,dgrad --iters 10 --batch 64 > gpurun_out/kbench_onebar.jsonl 2>gpurun_out/kbench.err
