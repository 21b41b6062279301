#!/bin/bash
# 8-stage LDS ring for one 64-tile GEMM block per CU: numerics, graph-timed kernel A/B, step A/B
set -o pipefail
O=gpurun_out/r4ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gemm or linear" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/kbench_gemm_small.py > $O/kg.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
cat $O/kg.jsonl
for i in 1 2; do for d in 1 0; do
  D3D_GEMM_DEEP8=$d timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_${d}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;print('deep8=$d b16',json.load(open('$O/b16_${d}_$i.json'))['value'])"
done; done
for d in 1 0; do
  D3D_GEMM_DEEP8=$d timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_${d}.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  python -c "import json;print('deep8=$d b128',json.load(open('$O/b128_${d}.json'))['value'])"
done
