#!/bin/bash
# kernel times inside the "L0 dec" flush batch (halo on / off)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r4n
mkdir -p $O
for h in 1 0; do
  for ex in 128 16; do
    D3D_WGRAD_HALO=$h timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/h${h}_e$ex -o run -- python3 /root/repo/tools/kbench_wgrad_group.py --examples $ex --only "L0 dec" --skip_old --iters 5 > $O/h${h}_e$ex.log 2>&1 || { tail $O/h${h}_e$ex.log; exit 1; }
    f=$(find $O/h${h}_e$ex -name '*kernel_stats.csv' | head -n1); echo "== h$h e$ex"; head -6 $f | cut -c1-200
  done
done
