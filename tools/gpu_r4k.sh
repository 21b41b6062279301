#!/bin/bash
# all-taps halo weight-gradient tiles: numerics, then A/B on the flush batches and the step
set -o pipefail
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad_group" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for ex in 128 16; do
  for h in 0 1 1,512,3 1,256,2 1,1024,2; do
    D3D_WGRAD_HALO=$h timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old > $O/h${h}_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  done
done
for f in $O/*.jsonl; do echo "== $f"; cut -c1-110 $f; done
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "graph_step_bitwise or full_model or graph_train_step or model_hip_vs" > $O/pytest2.log 2>&1 || { tail -30 $O/pytest2.log; exit 1; }
tail -2 $O/pytest2.log
for h in 1 0; do
  D3D_WGRAD_HALO=$h timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_h$h.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  D3D_WGRAD_HALO=$h timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_h$h.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  python -c "import json;[print('$h',f,json.load(open('$O/'+f+'_h$h.json'))['value']) for f in ('b16','b128')]"
done
