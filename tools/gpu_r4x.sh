#!/bin/bash
# 32-wide images on the halo conv (16-row tiles): numerics with it forced on, kernel A/B, step A/B
set -o pipefail
O=gpurun_out/r4x
mkdir -p $O
D3D_HALO_AU=5 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv3x3 or full_model" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for au in 5 1; do
  D3D_HALO_AU=$au timeout -k 10 200 python tools/kbench_conv_levels.py 256 > $O/kc_$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  D3D_HALO_AU=$au KB_CONV_EXTRA=1 timeout -k 10 200 python tools/kbench_conv_levels.py 256 >> $O/kc_$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== au$au"; grep '"32x32' $O/kc_$au.jsonl | cut -c1-220
done
for i in 1 2; do for au in 5 1; do
  D3D_HALO_AU=$au timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_${au}_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  python -c "import json;print('au$au b128', json.load(open('$O/b128_${au}_$i.json'))['value'])"
done; done
