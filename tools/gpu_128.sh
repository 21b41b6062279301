# 128x128 config (BASELINE config 4) on one GPU: global batch 128 in micro-batches of 32
set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python bench.py --imgsize 128 --micro_batch 32 --steps 4 --warmup 2 > $O/b128px.json 2> $O/b128px.err
rc=$?; tail -3 $O/b128px.err; cat $O/b128px.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 4 --global_batch 16 > $O/b16a.json 2>/dev/null || exit $?
cut -c1-400 $O/b16a.json
