# bs16 (the 8-GPU per-GPU share) steady-state trace: rocprofv3 kernel trace of
# 20 replayed steps; rpstats over the last 5 steps: per-kernel stats with the
# kernel count, device busy share and idle gaps.  Summaries under gpurun_out/p16.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/p16
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/db -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --global_batch 16 > $O/bench.log 2>&1
rc=$?
tail -n1 $O/bench.log | cut -c1-200
db=$(find $O/db -name '*.db' | head -n1)
if [ -n "$db" ]; then
  W=${WIN:-140}
  python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 5 --top 70 > $O/stats.txt
  python3 /root/repo/tools/rpstats.py "$db" --busy $W > $O/busy.txt
  python3 /root/repo/tools/rpstats.py "$db" --gaps $W --top 25 > $O/gaps.txt
  python3 /root/repo/tools/rpstats.py "$db" --solo $W --top 40 > $O/solo.txt
  find $O/db -name '*.db' -delete
fi
head -3 $O/stats.txt; cat $O/busy.txt | head -5; head -8 $O/gaps.txt
exit $rc
