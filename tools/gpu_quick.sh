set -o pipefail
cd /root/repo
O=/root/repo/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 15 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 --graph 1 > $O/b16.json 2>/dev/null || exit $?
echo "b16g $(cut -c1-170 $O/b16.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rpq -o run -- python3 /root/repo/bench.py --steps 6 --warmup 2 --global_batch 16 > $O/rpq.log 2>&1 || exit $?
db=$(find $O/rpq -name '*.db' | head -n1); python3 /root/repo/tools/rpstats.py "$db" --steps 8 --top 40 > $O/rpq_stats.txt; find $O/rpq -name '*.db' -delete
grep -E "pack_all|adam" $O/rpq_stats.txt
