#!/bin/bash
# halo conv AU at 128-wide images: numerics, kernel A/B, 128px bs16 graph-step A/B
set -o pipefail
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "conv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for au in 1 0; do
  D3D_HALO_AU=$au KB_CONV_128=1 timeout -k 10 200 python tools/kbench_conv_levels.py 32 > $O/kc128_au$au.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== au$au"; cat $O/kc128_au$au.jsonl
done
for au in 1 0; do
  D3D_HALO_AU=$au timeout -k 10 400 python bench.py --imgsize 128 --global_batch 16 --steps 10 --warmup 3 > $O/g16_au$au.json 2> $O/g16.err || { tail $O/g16.err; exit 1; }
  python -c "import json;print('au$au g16', json.load(open('$O/g16_au$au.json'))['value'])"
done
