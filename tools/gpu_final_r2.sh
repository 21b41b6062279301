# End-of-session evidence: smoke, headline benches (bs128 / bs16 / bs32 / 128x128 / sampling) and rocprofv3
# kernel traces of the bs128 and bs16 steps (window = last 10 steps; per-kernel, per-grid, solo and gap views)
set -o pipefail
cd /root/repo
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench128.json 2> $O/bench128.err || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/bench16.json 2> $O/bench16.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --global_batch 32 > $O/bench32.json 2> $O/bench32.err || exit $?
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --imgsize 128 > $O/bench128px.json 2> $O/bench128px.err || exit $?
timeout -k 10 400 python bench.py --mode sample > $O/sample.json 2> $O/sample.err || exit $?
for f in bench128 bench16 bench32 bench128px sample; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['unit'],d['ms_per_step'])"; done
BS="128 16" TAG=final/prof bash tools/gpu_prof16.sh
