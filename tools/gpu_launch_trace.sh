# hipGraphLaunch timing vs kernel trace at bs16 (graph replay)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/lt
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/db -o run -- python3 /root/repo/bench.py --steps 12 --warmup 3 --global_batch 16 > $O/b16.log 2>&1 || exit $?
db=$(find $O/db -name '*.db' | head -n1)
python3 /root/repo/tools/graph_launch_trace.py "$db" 8 > $O/launch.txt 2>&1
find $O/db -name '*.db' -delete
cat $O/launch.txt
