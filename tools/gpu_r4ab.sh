#!/bin/bash
# P2 halo conv (one barrier per tap pair, 8-slot weight ring): numerics forced on, kernel A/B, step A/B
set -o pipefail
O=gpurun_out/r4ab
mkdir -p $O
D3D_HALO_AU=61 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv3x3 or full_model or halo" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for au in 61 29; do
  D3D_HALO_AU=$au timeout -k 10 200 python tools/kbench_conv_levels.py 256 32 > $O/kc_$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  D3D_HALO_AU=$au KB_CONV_EXTRA=1 timeout -k 10 200 python tools/kbench_conv_levels.py 256 32 >> $O/kc_$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== au$au"; cut -c1-160 $O/kc_$au.jsonl
done
for i in 1 2; do for au in 61 29; do
  D3D_HALO_AU=$au timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_${au}_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  D3D_HALO_AU=$au timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_${au}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;[print('au$au',f,json.load(open('$O/'+f+'_${au}_$i.json'))['value']) for f in ('b128','b16')]"
done; done
