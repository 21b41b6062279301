# rocprofv3 kernel-trace of the training bench at global batch 128 and 16 (1 GPU);
# the rocpd databases are summarised on the box (tools/rpstats.py) and deleted.
# bs128 runs with the weight-gradient side stream off so per-kernel times are not
# inflated by concurrent kernels (ops/gradsink.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out
D3D_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rp128 -o run -- python3 /root/repo/bench.py --steps 6 --warmup 2 > $O/rp128.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rp16 -o run -- python3 /root/repo/bench.py --steps 10 --warmup 2 --global_batch 16 > $O/rp16.log 2>&1
rc=$?
tail -n1 $O/rp128.log | cut -c1-150; tail -n1 $O/rp16.log | cut -c1-150
for d in rp128 rp16; do
  db=$(find $O/$d -name '*.db' | head -n1)
  st=$([ $d = rp128 ] && echo 8 || echo 12)
  [ -n "$db" ] && python3 /root/repo/tools/rpstats.py "$db" --steps $st --top 80 > $O/${d}_stats.txt && \
    python3 /root/repo/tools/rpstats.py "$db" --steps $st --top 120 --grid > $O/${d}_grid.txt
  find $O/$d -name '*.db' -delete
done
du -sh $O/rp128 $O/rp16
exit $rc
