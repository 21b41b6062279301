# Full GPU verification of the tree: GPU test suite, smoke(), headline bench (bs128),
# per-GPU-share bench (bs16), graph-replay bench and the sampling bench.
set -o pipefail
cd /root/repo
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench128.json 2> $O/bench128.err || exit $?
cat $O/bench128.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/bench16.json 2> $O/bench16.err || exit $?
cat $O/bench16.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --graph 1 > $O/bench128g.json 2> $O/bench128g.err || exit $?
cat $O/bench128g.json
timeout -k 10 300 python bench.py --mode sample > $O/bench_sample.json 2> $O/bench_sample.err || exit $?
cat $O/bench_sample.json
