# rocpd kernel trace of a few bench steps (usage: bash tools/step_timeline.sh <out> <global_batch>)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $O/db -o run -- python3 $R/bench.py --steps 3 --warmup 2 --global_batch $2 > $O/run.log 2>&1
echo ok
