# round 4: bs128 eager weight-gradient paths (per-job kernels / deferred grouped / one-job grouped) and bs16
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
for rep in 1 2; do for g in 0 1 2; do
  D3D_WGRAD_EAGER_GROUP=$g timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_e${g}_$rep.json 2> $O/b128.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b128_e${g}_$rep.json'));print('b128 eager_group=$g', d['value'], d['ms_per_step'])"
done; done
timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16.json 2> $O/b16.err || exit $?
python3 -c "import json;d=json.load(open('$O/b16.json'));print('b16', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --global_batch 32 --steps 30 --warmup 5 > $O/b32.json 2> $O/b32.err || exit $?
python3 -c "import json;d=json.load(open('$O/b32.json'));print('b32', d['value'], d['ms_per_step'])"
