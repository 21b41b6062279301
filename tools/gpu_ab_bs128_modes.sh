# bs128 step-mode A/B: micro-batch size x HIP-graph replay (interleaved, two rounds)
set -o pipefail
cd /root/repo
O=gpurun_out/modes
mkdir -p $O
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'],d['config']['micro_batch'],d['config']['hip_graph'])"; }
for round in 1 2; do
  for cfg in "mb64_eager:--micro_batch 64 --graph 0" "mb64_graph:--micro_batch 64 --graph 1" "mb128_eager:--micro_batch 128 --graph 0" "mb128_graph:--micro_batch 128 --graph 1" "mb32_graph:--micro_batch 32 --graph 1"; do
    lab=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python bench.py --steps 12 --warmup 4 $args > $O/$lab.json 2> $O/$lab.err || exit $?
    echo "$lab $(show $O/$lab.json)"
  done
done
# FiLM weight-gradient path at bs128 (auto = hipBLASLt above 32 frames)
for round in 1 2; do
  for v in blas mfma; do
    D3D_FILM_WGRAD=$v timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/fw_$v.json 2> $O/fw_$v.err || exit $?
    echo "film_wgrad=$v $(show $O/fw_$v.json)"
  done
done
