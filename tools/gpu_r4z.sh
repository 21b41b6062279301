#!/bin/bash
# dense-GEMM tile / grouping knobs at bs16 (the small attention / NIN GEMMs are on the critical path there)
set -o pipefail
O=gpurun_out/r4z
mkdir -p $O
for i in 1 2; do for t in 0,0,0 4,0,0 2,0,0 0,4,0 0,16,0; do
  D3D_GEMM_TUNE=$t timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_${t}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;print('$t b16', json.load(open('$O/b16_${t}_$i.json'))['value'])"
done; done
