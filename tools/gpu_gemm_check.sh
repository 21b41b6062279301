# GEMM kernel iteration: numerics tests, then the shape microbenchmark.
set -o pipefail
cd /root/repo && export PYTHONPATH=/root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or linear or film_batch" > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_kgemm.sh
