set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/pp_prof
mkdir -p $O
B=16
export D3D_LIN_PP=1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --global_batch $B > $O/b.json 2> $O/b.err || exit $?
db=$(find $O/rp -name '*.db' | head -n1)
ms=$(python3 -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")
W=$(python3 -c "print(10*$ms)")
python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 10 --top 40 > $O/stats.txt
python3 /root/repo/tools/rpstats.py "$db" --solo $W --steps 10 --top 40 > $O/solo.txt
python3 /root/repo/tools/rpstats.py "$db" --window $W --steps 10 --top 200 --grid | grep -i gemm > $O/grid.txt || true
find $O/rp -name '*.db' -delete
