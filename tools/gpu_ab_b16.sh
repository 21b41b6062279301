# A/B an environment switch on the graph-replayed small-batch steps only
# (per-GPU batch 16 and 32: the 8- and 4-GPU shares of global batch 128):
#   bash tools/gpu_ab_b16.sh VAR V1 V2 [V3 ...]
set -o pipefail
cd /root/repo
O=gpurun_out
V=${1:?variable}; shift
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for round in 1 2; do
  for val in "$@"; do
    for bs in 16 32; do
      env $V=$val timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch $bs > $O/abs_${bs}_$val.json 2>$O/abs_${bs}_$val.err || exit $?
      echo "b$bs $V=$val $(show $O/abs_${bs}_$val.json)"
    done
  done
done
