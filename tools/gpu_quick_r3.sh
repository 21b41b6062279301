# quick check while iterating: selected GPU tests (-k "$K"), then the bs16 and bs128 benches
set -o pipefail
O=gpurun_out/quick
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16_$i.json 2> $O/b16.err || exit $?
python3 -c "import json;d=json.load(open('$O/b16_$i.json'));print('b16', d['value'], d['ms_per_step'])"
done
if [ -n "$B128" ]; then
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b128.json 2> $O/b128.err || exit $?
python3 -c "import json;d=json.load(open('$O/b128.json'));print('b128', d['value'], d['ms_per_step'])"
fi
