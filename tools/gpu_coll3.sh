set -o pipefail
for i in 1 2 3; do
  timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 150 --timeout-method thread -k "captured_collectives_one_rank or graph_capture_probe or two_ranks_one_gpu" > gpurun_out/coll_$i.log 2>&1 || { tail -5 gpurun_out/coll_$i.log; exit 1; }
  tail -1 gpurun_out/coll_$i.log
done
