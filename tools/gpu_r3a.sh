# round-3 working GPU check: determinism bisect, GN roofline, GPU suite, smoke, benches
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u tools/diag_determinism.py ${DIAG:-g:scd,g:scd,g:cd,g:cd,g:sd,g:sd,g:sc,g:sc,e:sc,e:sc} > $O/diag_det.txt 2>&1 || exit $?
timeout -k 10 300 python tools/kbench_gn.py > $O/kbench_gn.jsonl 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_ops_gpu.py::test_graph_step_bitwise_deterministic --deselect "tests/test_ops_gpu.py::test_fused_update_matches_separate[False]" > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench128.json 2> $O/bench128.err || exit $?
cat $O/bench128.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/bench16.json 2> $O/bench16.err || exit $?
cat $O/bench16.json
