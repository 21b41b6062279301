# bs16 eager vs HIP-graph step, repeated (host-jitter check)
set -o pipefail
cd /root/repo
O=gpurun_out
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --global_batch 16 > $O/b16e.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --global_batch 16 --graph 1 > $O/b16g.json 2>/dev/null || exit $?
echo "eager $(cut -c100-200 $O/b16e.json)"; echo "graph $(cut -c100-200 $O/b16g.json)"
done
nproc; cat /proc/loadavg
