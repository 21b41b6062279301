#!/bin/bash
# gradient zeroing folded into the fused Adam (graph step): graph == eager tests, bench
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "graph or adam" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  timeout -k 10 300 python bench.py --global_batch 32 --steps 20 --warmup 5 > $O/b32_$i.json 2> $O/b32.err || { tail $O/b32.err; exit 1; }
  python -c "import json;[print(f,json.load(open('$O/'+f+'_$i.json'))['value']) for f in ('b16','b32')]"
done
