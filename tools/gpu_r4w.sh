#!/bin/bash
# direct weight gradients (conditioning conv) on the halo tile: numerics + A/B
set -o pipefail
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad or cond_conv or full_model or model_hip_vs or conv3x3" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for d in 1 0; do
  D3D_WGRAD_DIRECT_HALO=$d timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_d${d}_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  D3D_WGRAD_DIRECT_HALO=$d timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_d${d}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;[print('d$d',f,json.load(open('$O/'+f+'_d${d}_$i.json'))['value']) for f in ('b128','b16')]"
done; done
