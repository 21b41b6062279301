# bs16 graph step under HIP runtime settings: host wait policy / queues (interleaved, 2 rounds)
set -o pipefail
O=gpurun_out/envab
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 0; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run base$r X=1
  run wait1s$r ROC_ACTIVE_WAIT_TIMEOUT=1000000
  run wait0$r ROC_ACTIVE_WAIT_TIMEOUT=0
  run hwq8_$r GPU_MAX_HW_QUEUES=8
  run hwq8w$r GPU_MAX_HW_QUEUES=8 ROC_ACTIVE_WAIT_TIMEOUT=1000000
  run hwq16_$r GPU_MAX_HW_QUEUES=16
done
