# targeted GPU tests of the deferred update + interleaved A/B of D3D_DEFER_UPDATE at bs16 / bs32
set -o pipefail
cd /root/repo
O=gpurun_out/defer
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "graph or fused_update or sink or determin" > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for v in 0 1; do
    D3D_DEFER_UPDATE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$v.json 2> $O/b16_$v.err || exit $?
    echo "b16 defer=$v $(show $O/b16_$v.json)"
    D3D_DEFER_UPDATE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --global_batch 32 > $O/b32_$v.json 2> $O/b32_$v.err || exit $?
    echo "b32 defer=$v $(show $O/b32_$v.json)"
  done
done
