# Quick GPU check used while iterating: a pytest selection (-k "$K"), then the
# per-GPU-batch 16 and 128 benches.  Outputs under gpurun_out/$TAG.
set -o pipefail
O=gpurun_out/${TAG:-quick}
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 150 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/b16.json 2> $O/b16.err || exit $?
timeout -k 10 150 python bench.py --global_batch 32 --steps 20 --warmup 5 > $O/b32.json 2> $O/b32.err || exit $?
[ -n "$B128" ] && { timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/b128.json 2> $O/b128.err || exit $?; }
for f in $O/b*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['value'],d['ms_per_step'])"; done
