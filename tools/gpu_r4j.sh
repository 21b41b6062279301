#!/bin/bash
# grouped weight-gradient: LDS ring depth / wide-tile re-check at bs128 and bs16 shapes
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
for ex in 128 16; do
  for ns in 2 3 4; do
    D3D_WGRAD_GROUP_NS=$ns timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old > $O/ns${ns}_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
  done
  D3D_WGRAD_GROUP_WIDE=1 timeout -k 10 120 python tools/kbench_wgrad_group.py --examples $ex --skip_old > $O/wide_e$ex.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
done
for f in $O/*.jsonl; do echo "== $f"; cut -c1-120 $f; done
