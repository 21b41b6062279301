#!/bin/bash
# sigmoid via v_rcp_f32: numerics (GN / FiLM / conv SiLU users), kernel-family and step A/B against the
# previous build (D3D_LIB_PATH=build/ab/009325d/libd3d_hip.so)
set -o pipefail
O=gpurun_out/r4ae
mkdir -p $O
REF=build/ab/009325d/libd3d_hip.so
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gn or silu or film or gemm or full_model or cond" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_new_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  D3D_LIB_PATH=$REF timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_ref_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_new_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  D3D_LIB_PATH=$REF timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_ref_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  for v in new ref; do python -c "import json;[print('$v',f,json.load(open('$O/'+f+'_${v}_$i.json'))['value']) for f in ('b128','b16')]"; done
done
