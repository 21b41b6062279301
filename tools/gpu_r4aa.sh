#!/bin/bash
# halo weight gradient with 64-pixel K-steps on W >= 64 jobs: numerics, flush batches, bench A/B
set -o pipefail
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "wgrad_group" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pk in 64 32; do for ex in 128 16; do
  D3D_WGRAD_HALO_PK=$pk timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old --only L0 > $O/kb_pk${pk}_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  echo "== pk$pk e$ex"; cut -c1-100 $O/kb_pk${pk}_e$ex.jsonl
done; done
for i in 1 2; do for pk in 64 32; do
  D3D_WGRAD_HALO_PK=$pk timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/b128_pk${pk}_$i.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
  D3D_WGRAD_HALO_PK=$pk timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16_pk${pk}_$i.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
  python -c "import json;[print('pk$pk',f,json.load(open('$O/'+f+'_pk${pk}_$i.json'))['value']) for f in ('b128','b16')]"
done; done
