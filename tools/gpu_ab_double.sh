# two executables of the step graph replayed alternately (D3D_GRAPH_DOUBLE): graph tests + bs16/bs32 A/B
set -o pipefail
cd /root/repo
O=gpurun_out/dbl
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 300 --timeout-method thread -k "graph or fused_update" > $O/tests.log 2>&1
rc=$?; tail -n 3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'],d['hbm_peak_gib'])"; }
for r in 1 2; do
  for v in 0 1; do
    D3D_GRAPH_DOUBLE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16_$v.json 2> $O/b16_$v.err || exit $?
    echo "b16 double=$v $(show $O/b16_$v.json)"
    D3D_GRAPH_DOUBLE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --global_batch 32 > $O/b32_$v.json 2> $O/b32_$v.err || exit $?
    echo "b32 double=$v $(show $O/b32_$v.json)"
  done
done
# bs64 (the 2-GPU share): graph step (deferred update, alternate executables) vs the eager step
for r in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --steps 15 --warmup 4 --global_batch 64 --graph $g > $O/b64_g$g.json 2> $O/b64_g$g.err || exit $?
    echo "b64 graph=$g $(show $O/b64_g$g.json)"
  done
done
