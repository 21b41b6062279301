# GPU test suite + headline benches (bs128 / bs16) + bs16 gap attribution
set -o pipefail
cd /root/repo
O=gpurun_out/vq
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_$r.json 2> $O/b128_$r.err || exit $?
  echo "b128 $(show $O/b128_$r.json)"
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$r.json 2> $O/b16_$r.err || exit $?
  echo "b16  $(show $O/b16_$r.json)"
done
BS=16 TAG=vq/prof bash tools/gpu_prof16.sh && head -8 $O/prof/bs16_gaps.txt
