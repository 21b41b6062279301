set -o pipefail
O=gpurun_out/fws; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "film_batch" -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do for v in 1 0; do
  D3D_FILM_WGRAD_SPLIT=$v timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_$v.json 2>$O/b128_$v.err || exit $?
  echo "b128 split=$v $(show $O/b128_$v.json)"
  D3D_FILM_WGRAD_SPLIT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 4 --global_batch 32 > $O/b32_$v.json 2>$O/b32_$v.err || exit $?
  echo "b32  split=$v $(show $O/b32_$v.json)"
done; done
