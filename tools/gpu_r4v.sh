#!/bin/bash
# GroupNorm blocks per launch at bs16 / bs32 end to end (D3D_GN_CFG), alternating
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
for i in 1 2; do for c in 512,1,2 1024,1,2; do
  D3D_GN_CFG=$c timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_${c}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  D3D_GN_CFG=$c timeout -k 10 300 python bench.py --global_batch 32 --steps 20 --warmup 5 > $O/b32_${c}_$i.json 2> $O/b32.err || { tail $O/b32.err; exit 1; }
  python -c "import json;[print('$c',f,json.load(open('$O/'+f+'_${c}_$i.json'))['value']) for f in ('b16','b32')]"
done; done
