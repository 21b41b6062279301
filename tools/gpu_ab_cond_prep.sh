# conditioning-prep + per-block FiLM event: targeted tests, then bs16 / bs128 benches vs the previous commit's
# numbers (profiles/ab_defer_update_r2.txt); two rounds
set -o pipefail
cd /root/repo
O=gpurun_out/cp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "ray or cond or graph or oracle or posenc or determin" > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$r.json 2> $O/b16_$r.err || exit $?
  echo "b16  $(show $O/b16_$r.json)"
  timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/b128_$r.json 2> $O/b128_$r.err || exit $?
  echo "b128 $(show $O/b128_$r.json)"
done
