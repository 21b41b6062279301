# bs128 one-micro-batch: grid-target knobs chosen at micro-batch 64, re-checked (ex/s ms/step, two interleaved rounds)
set -o pipefail
cd /root/repo
O=gpurun_out/knobs
mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for cfg in "base:" "wt512:D3D_WGRAD_TARGET=512" "wt2048:D3D_WGRAD_TARGET=2048" "gn2048:D3D_GN_TARGET=2048" "gn512:D3D_GN_TARGET=512" "halo32:D3D_HALO32=1"; do
    lab=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 4 > $O/$lab.json 2> $O/$lab.err || exit $?
    echo "$lab $(show $O/$lab.json)"
  done
done
