# kernel traces of the slow 128x128 variants (one micro-batch of 128; conditioning stream at 64)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/p128px
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/dba -o run -- python3 /root/repo/bench.py --imgsize 128 --steps 2 --warmup 1 --micro_batch 0 > $O/a.log 2>&1 || exit $?
D3D_COND_STREAM=2 timeout -k 10 500 rocprofv3 --kernel-trace -d $O/dbb -o run -- python3 /root/repo/bench.py --imgsize 128 --steps 2 --warmup 1 > $O/b.log 2>&1 || exit $?
for d in a b; do
  db=$(find $O/db$d -name '*.db' | head -n1)
  python3 /root/repo/tools/rpstats.py "$db" --window 3000 --top 25 --grid > $O/grid_$d.txt
  python3 /root/repo/tools/rpstats.py "$db" --busy 3000 > $O/busy_$d.txt
  find $O/db$d -name '*.db' -delete
done
head -14 $O/grid_a.txt; cat $O/busy_a.txt; head -14 $O/grid_b.txt; cat $O/busy_b.txt
