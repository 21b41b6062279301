# stream priorities: weight-gradient stream / conditioning stream, bs16 + bs128, two interleaved rounds
set -o pipefail
cd /root/repo
O=gpurun_out/prio
mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for cfg in "base:" "wg_hi:D3D_WGRAD_STREAM_PRIO=-1" "cs_hi:D3D_COND_STREAM_PRIO=-1" "both_hi:D3D_WGRAD_STREAM_PRIO=-1 D3D_COND_STREAM_PRIO=-1"; do
    lab=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$lab.json 2> $O/b16_$lab.err || exit $?
    echo "b16  $lab $(show $O/b16_$lab.json)"
  done
done
for r in 1 2; do
  for cfg in "base:" "wg_hi:D3D_WGRAD_STREAM_PRIO=-1"; do
    lab=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/b128_$lab.json 2> $O/b128_$lab.err || exit $?
    echo "b128 $lab $(show $O/b128_$lab.json)"
  done
done
