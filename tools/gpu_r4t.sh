#!/bin/bash
# halo conv AU with the residual preloaded into the accumulators: numerics, kernel A/B, bench A/B
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv or full_model or model_hip_vs or residual or graph_step_bitwise" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for au in 1 0; do
  D3D_HALO_AU=$au timeout -k 10 200 python tools/kbench_conv_levels.py 256 32 > $O/kc_au$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== au$au"; grep '64x64' $O/kc_au$au.jsonl
done
for i in 1 2; do for au in 1 0; do
  D3D_HALO_AU=$au timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_au${au}_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  D3D_HALO_AU=$au timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_au${au}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;[print('au$au',f,json.load(open('$O/'+f+'_au${au}_$i.json'))['value']) for f in ('b128','b16')]"
done; done
