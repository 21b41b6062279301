#!/bin/bash
# halo wgrad with the whole-round planner: numerics, flush batches, step A/B
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad_group" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for ex in 128 16; do
  for h in 1 1,512,2; do
    D3D_WGRAD_HALO=$h timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old > $O/h${h}_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
    echo "== h$h e$ex"; cut -c1-100 $O/h${h}_e$ex.jsonl
  done
done
for h in 1 0 1 0; do
  D3D_WGRAD_HALO=$h timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_h$h.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  D3D_WGRAD_HALO=$h timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_h$h.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  python -c "import json;[print('$h',f,json.load(open('$O/'+f+'_h$h.json'))['value']) for f in ('b16','b128')]"
done
