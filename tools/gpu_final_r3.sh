# end-of-round evidence: GPU suite, smoke, headline + per-GPU-share + sampling benches,
# rocprofv3 traces (bs128, bs16) summarised on the box
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench128.json 2> $O/bench128.err || exit $?
cat $O/bench128.json
timeout -k 10 300 python bench.py --steps 40 --warmup 8 --global_batch 16 > $O/bench16.json 2> $O/bench16.err || exit $?
cat $O/bench16.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 32 > $O/bench32.json 2> $O/bench32.err || exit $?
cat $O/bench32.json
timeout -k 10 300 python bench.py --mode sample > $O/sample.json 2> $O/sample.err || exit $?
cat $O/sample.json
[ -n "$PROF" ] && { bash tools/gpu_prof_r3.sh > $O/prof.log 2>&1 || exit $?; }
[ -n "$PROF" ] && tail -12 $O/prof.log; true
