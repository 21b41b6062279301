# 128x128: allocator configuration vs one micro-batch of 128 / conditioning stream; 64x64 regressions
set -o pipefail
O=gpurun_out/b128px
mkdir -p $O
run() {  # name, env, args
  local name=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 400 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d['hbm_peak_gib'], d.get('alloc_retries'))"
}
E=PYTORCH_HIP_ALLOC_CONF=expandable_segments:True
run x_mb128 $E --imgsize 128 --steps 6 --warmup 2 --micro_batch 0 || exit 1
run x_mb64 $E --imgsize 128 --steps 6 --warmup 2 || exit 1
run x_mb128cond "$E D3D_COND_STREAM=2" --imgsize 128 --steps 6 --warmup 2 --micro_batch 0 || exit 1
run x_b16 $E --global_batch 16 --steps 30 --warmup 5 || exit 1
run b16 X=1 --global_batch 16 --steps 30 --warmup 5 || exit 1
run x_b128 $E --steps 15 --warmup 4 || exit 1
run b128 X=1 --steps 15 --warmup 4 || exit 1
