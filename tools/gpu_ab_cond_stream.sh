# GPU suite (conditioning stream on) + interleaved A/B of D3D_COND_STREAM at bs16 / bs128
set -o pipefail
cd /root/repo
O=gpurun_out/cs
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for v in 0 1; do
    D3D_COND_STREAM=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$v.json 2> $O/b16_$v.err || exit $?
    echo "b16  cond_stream=$v $(show $O/b16_$v.json)"
    D3D_COND_STREAM=$v timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/b128_$v.json 2> $O/b128_$v.err || exit $?
    echo "b128 cond_stream=$v $(show $O/b128_$v.json)"
  done
done
