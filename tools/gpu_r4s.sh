#!/bin/bash
# flat split reduce for 1x1 jobs: numerics, flush batches, bench
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad or full_model or graph_step_bitwise or linear or cat_gn" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ex in 16 128; do
  timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old > $O/kb_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== e$ex"; cut -c1-100 $O/kb_e$ex.jsonl
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  python -c "import json;[print(f,json.load(open('$O/'+f+'_$i.json'))['value']) for f in ('b16','b128')]"
done
