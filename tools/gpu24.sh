set -o pipefail
cd /root/repo
timeout -k 10 900 python -m pytest tests/test_ops_gpu.py -x -q -k "conv or model or graph" > gpurun_out/test_conv.log 2>&1
rc=$?; tail -3 gpurun_out/test_conv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py --ops conv,dgrad --iters 10 --batch 64 > gpurun_out/kbench_bufl.jsonl 2>gpurun_out/kbench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d /root/repo/gpurun_out/pmc5 -o run -- python3 /root/repo/tools/kbench.py --ops conv,dgrad --iters 2 --batch 64 > /root/repo/gpurun_out/pmc5.log 2>&1
