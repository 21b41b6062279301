# A/B(/C...) an environment switch on the headline benches:
#   bash tools/gpu_ab_env.sh [--tests] VAR V1 V2 [V3 ...]
# runs bs128 and bs16 for every value, two interleaved rounds; --tests runs the
# full GPU test suite first.
set -o pipefail
cd /root/repo
O=gpurun_out
if [ "$1" = --tests ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
V=${1:?variable}; shift
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for round in 1 2; do
  for val in "$@"; do
    env $V=$val timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/ab128_$val.json 2>$O/ab128_$val.err || exit $?
    echo "b128 $V=$val $(show $O/ab128_$val.json)"
    env $V=$val timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/ab16_$val.json 2>$O/ab16_$val.err || exit $?
    echo "b16  $V=$val $(show $O/ab16_$val.json)"
  done
done
