# GPU occupancy of the bs16 graph step with the weight-gradient side stream on/off
# (rocprofv3 kernel trace; union of kernel intervals over the last 200 ms)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out
for v in 1 0; do
  D3D_WGRAD_STREAM=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/bz$v -o run -- python3 /root/repo/bench.py --steps 10 --warmup 3 --global_batch 16 > $O/bz$v.log 2>&1 || exit $?
  db=$(find $O/bz$v -name '*.db' | head -n1)
  echo "stream=$v $(python3 /root/repo/tools/rpstats.py "$db" --busy 200)"
  python3 /root/repo/tools/rpstats.py "$db" --steps 13 --top 60 > $O/bz${v}_stats.txt
  find $O/bz$v -name '*.db' -delete
done
