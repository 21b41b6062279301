#!/bin/bash
# GroupNorm launch shapes at bs16 (N=32 frames), device times from rocprofv3 kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/gn16
mkdir -p $O
for c in 1024,1,2 1024,2,2 2048,1,2 2048,2,4 4096,2,2 512,1,2; do
  D3D_GN_CFG=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/c$c -o run --output-format csv -- python3 /root/repo/tools/kbench_gn.py 32 > $O/c$c.log 2>&1 || exit 1
  f=$(find $O/c$c -name '*kernel_stats.csv' | head -n1)
  echo "== $c"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "gn_" in r["Name"]:
        print("  %-60s n=%5s avg=%8.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf $O/c$c
done
