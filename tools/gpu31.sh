set -o pipefail
cd /root/repo
for v in 0 1 0 1; do
  D3D_CAT_FUSE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/ab16_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab16_$v.log').read().strip().splitlines()[-1]);print('bs16 fuse=$v', d['value'], d['ms_per_step'])"
done
for v in 0 1; do
  D3D_CAT_FUSE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('bs128 fuse=$v', d['value'], d['ms_per_step'])"
done
