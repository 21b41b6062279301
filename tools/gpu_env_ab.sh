# GPU_MAX_HW_QUEUES 4 (box default) vs 8 at bs16 and bs128, interleaved
set -o pipefail
O=gpurun_out/envab
mkdir -p $O
run() {
  local name=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 300 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run b16_q4_$r X=1 --global_batch 16 --steps 40 --warmup 8 || exit 1
  run b16_q8_$r GPU_MAX_HW_QUEUES=8 --global_batch 16 --steps 40 --warmup 8 || exit 1
  run b128_q4_$r X=1 --steps 15 --warmup 4 || exit 1
  run b128_q8_$r GPU_MAX_HW_QUEUES=8 --steps 15 --warmup 4 || exit 1
done
