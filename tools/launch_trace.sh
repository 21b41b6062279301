set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lt; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format rocpd -d $O/db -o run -- python3 $R/bench.py --steps 8 --warmup 4 --global_batch 16 > $O/run.log 2>&1
ls -R $O/db | head
DB=$(find $O/db -name "*.db" | head -1)
python3 $R/tools/graph_launch_trace.py "$DB" 6 > $O/lt.txt 2>&1
echo ok
