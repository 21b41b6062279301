# 128x128 one micro-batch of 128 under caching-allocator settings
set -o pipefail
O=gpurun_out/b128px
mkdir -p $O
run() {  # name, env, args
  local name=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 400 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'], d['hbm_peak_gib'], d.get('alloc_retries'))"
}
run gc80 PYTORCH_HIP_ALLOC_CONF=garbage_collection_threshold:0.8 --imgsize 128 --steps 6 --warmup 2 --micro_batch 0 || exit 1
run gc60 PYTORCH_HIP_ALLOC_CONF=garbage_collection_threshold:0.6 --imgsize 128 --steps 6 --warmup 2 --micro_batch 0 || exit 1
run split PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:1024 --imgsize 128 --steps 6 --warmup 2 --micro_batch 0 || exit 1
run gc80cond "PYTORCH_HIP_ALLOC_CONF=garbage_collection_threshold:0.8 D3D_COND_STREAM=2" --imgsize 128 --steps 6 --warmup 2 || exit 1
