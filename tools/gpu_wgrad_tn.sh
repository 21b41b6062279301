# TN weight-gradient GEMM: numerics tests, then the FiLM-shape microbenchmark.
set -o pipefail
cd /root/repo && export PYTHONPATH=/root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad_tn or film_batch" > gpurun_out/wgrad_tn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wgrad_tn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kbench_wgrad_tn.py 2>&1 | tee gpurun_out/kbench_wgrad_tn.jsonl
