# rocprofv3 kernel trace of the steady-state graph step at per-GPU batch 16 and 32
# (the 8- and 4-GPU shares of the global batch 128): per-kernel ms/step over the
# last STEPS steps only (tools/rpstats.py --window), plus per-grid rows.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/${TAG:-prof}
mkdir -p $O
for B in ${BS:-16 32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp$B -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --global_batch $B > $O/b$B.json 2> $O/b$B.err || exit $?
  db=$(find $O/rp$B -name '*.db' | head -n1)
  ms=$(python3 -c "import json;print(json.load(open('$O/b$B.json'))['ms_per_step'])")
  W=$(python3 -c "print(10*$ms)")
  python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 10 --top 90 > $O/bs${B}_stats.txt
  python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 10 --top 160 --grid > $O/bs${B}_grid.txt
  python3 /root/repo/tools/rpstats.py "$db" --busy $W >> $O/bs${B}_stats.txt
  python3 /root/repo/tools/rpstats.py "$db" --solo $W --steps 10 --top 60 > $O/bs${B}_solo.txt
  python3 /root/repo/tools/rpstats.py "$db" --gaps $W --steps 10 --top 40 > $O/bs${B}_gaps.txt
  find $O/rp$B -name '*.db' -delete
done
