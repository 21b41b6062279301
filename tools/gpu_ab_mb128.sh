# bs128 as ONE micro-batch (bench default since ab_bs128_modes_r2): env A/B of the switches whose
# defaults were chosen at micro-batch 64
set -o pipefail
cd /root/repo
O=gpurun_out/mb128
mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'],d['config']['micro_batch'],d.get('hbm_peak_gib'))"; }
for round in 1 2; do
  for cfg in "base:" "fw_mfma:D3D_FILM_WGRAD=mfma" "linpp:D3D_LIN_PP=1" "nows:D3D_WGRAD_STREAM=0"; do
    lab=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/$lab.json 2> $O/$lab.err || exit $?
    echo "$lab $(show $O/$lab.json)"
  done
done
