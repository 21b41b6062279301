set -o pipefail
cd /root/repo && export PYTHONPATH=/root/repo
mkdir -p gpurun_out
timeout -k 10 300 python tools/kbench_gemm.py ${ONLY:+--only "$ONLY"} --vers ${VERS:-1} --rounds 3 --iters 20 > gpurun_out/kg_v3.jsonl 2> gpurun_out/kg_v3.err
rc=$?
cat gpurun_out/kg_v3.jsonl; tail -5 gpurun_out/kg_v3.err
exit $rc
