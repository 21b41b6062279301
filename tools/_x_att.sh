set -o pipefail
mkdir -p gpurun_out/r6_att
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or attn or full_model or graph_train_step or bitwise" > gpurun_out/r6_att/tests.log 2>&1 || { tail -40 gpurun_out/r6_att/tests.log; exit 1; }
tail -1 gpurun_out/r6_att/tests.log
