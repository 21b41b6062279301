# round-3 check after the GEMM LDS-race fix: concurrency screen, determinism,
# GPU suite, smoke, headline and per-GPU-share benches
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u tools/stress_concurrent.py 24 > $O/stress.txt 2>&1 || exit $?
grep -v "mismatches 0/" $O/stress.txt | grep -v amdgpu.ids
timeout -k 10 400 python -u tools/diag_determinism.py e:sc,e:sc,e:sc,e:sc,g:scd,g:scd,g:scd,g:scd > $O/diag_det.txt 2>&1 || exit $?
grep "losses equal" $O/diag_det.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench128.json 2> $O/bench128.err || exit $?
cat $O/bench128.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/bench16.json 2> $O/bench16.err || exit $?
cat $O/bench16.json
