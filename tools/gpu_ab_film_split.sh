# level-batched FiLM forward split (first block's columns first, one shared output): smoke + model/graph tests + A/B
set -o pipefail
cd /root/repo
O=gpurun_out/fs
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "film or graph or oracle or model or sampler" > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for v in 0 1; do
    D3D_FILM_SPLIT_FIRST=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$v.json 2> $O/b16_$v.err || exit $?
    echo "b16  split=$v $(show $O/b16_$v.json)"
    D3D_FILM_SPLIT_FIRST=$v timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/b128_$v.json 2> $O/b128_$v.err || exit $?
    echo "b128 split=$v $(show $O/b128_$v.json)"
  done
done
