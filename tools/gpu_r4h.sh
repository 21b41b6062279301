#!/bin/bash
# GroupNorm backward launch-shape sweep (tools/kbench_gn.py)
set -o pipefail
mkdir -p gpurun_out/r4h
for c in 1024,1,2 2048,1,2 4096,1,2 1024,2,2 1024,1,4 2048,2,4 512,1,2 2048,1,1; do
  D3D_GN_CFG=$c timeout -k 10 150 python tools/kbench_gn.py 32 256 > gpurun_out/r4h/gn_$c.jsonl 2> gpurun_out/r4h/gn_$c.err || exit 1
  echo "done $c"
done
