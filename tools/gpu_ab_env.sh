# A/B an environment switch on the headline benches:
#   bash tools/gpu_ab_env.sh VAR A B [tests]   (VAR=A vs VAR=B, bs128 and bs16, twice, interleaved;
#   "tests": run the full GPU test suite first)
set -o pipefail
cd /root/repo
O=gpurun_out
V=${1:?variable}; A=${2:?value A}; B=${3:?value B}
if [ "${4:-}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for val in $A $B $A $B; do
  env $V=$val timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/ab128_$val.json 2>$O/ab128_$val.err || exit $?
  echo "b128 $V=$val $(python3 -c "import json;d=json.load(open('$O/ab128_$val.json'));print(d['value'],d['ms_per_step'])")"
  env $V=$val timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/ab16_$val.json 2>$O/ab16_$val.err || exit $?
  echo "b16  $V=$val $(python3 -c "import json;d=json.load(open('$O/ab16_$val.json'));print(d['value'],d['ms_per_step'])")"
done
