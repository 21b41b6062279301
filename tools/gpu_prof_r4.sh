# rocprofv3 kernel traces of the training bench at the headline config (bs128)
# and the 8-GPU per-GPU share (bs16, graph replay), production settings (side
# streams on); rpstats summaries (stats, grid, exposed/solo, gaps) on the box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/${PROF_OUT:-prof5}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/db128 -o run -- python3 /root/repo/bench.py --steps 8 --warmup 3 > $O/b128.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/db16 -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --global_batch 16 > $O/b16.log 2>&1 || exit $?
for d in 128 16; do
  db=$(find $O/db$d -name '*.db' | head -n1)
  st=$([ $d = 128 ] && echo 8 || echo 20)
  W=$([ $d = 128 ] && echo 670 || echo 140)
  python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 5 --top 80 > $O/stats$d.txt
  python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 5 --top 120 --grid > $O/grid$d.txt
  python3 /root/repo/tools/rpstats.py "$db" --busy $W > $O/busy$d.txt
  python3 /root/repo/tools/rpstats.py "$db" --gaps $W --top 25 > $O/gaps$d.txt
  python3 /root/repo/tools/rpstats.py "$db" --solo $W --top 50 > $O/solo$d.txt
  find $O/db$d -name '*.db' -delete
done
tail -n1 $O/b128.log | cut -c1-150; tail -n1 $O/b16.log | cut -c1-150
head -3 $O/stats128.txt; head -3 $O/stats16.txt; cat $O/busy16.txt | head -4; head -5 $O/gaps16.txt
grep -c Cijk $O/stats128.txt $O/stats16.txt || true
python3 /root/repo/tools/famsum.py $O/stats128.txt > $O/families.txt; python3 /root/repo/tools/famsum.py $O/stats16.txt >> $O/families.txt; cat $O/families.txt
