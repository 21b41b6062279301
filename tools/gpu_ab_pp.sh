set -o pipefail
cd /root/repo
O=gpurun_out
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
run() { # label envs...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/ab128_$lab.json 2>$O/ab128_$lab.err || exit $?
  echo "b128 $lab $(show $O/ab128_$lab.json)"
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/ab16_$lab.json 2>$O/ab16_$lab.err || exit $?
  echo "b16  $lab $(show $O/ab16_$lab.json)"
}
for round in 1 2; do
  run off D3D_LIN_PP=0
  run persist D3D_LIN_PP=1
  run nonpersist D3D_LIN_PP=1 D3D_GEMM_GRID=100000000
done
