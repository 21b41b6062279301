# round 4: GroupNorm-backward partials from the halo dgrad epilogue -- numerics + bs16 / bs128 A/B
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "backward_partials or group_norm or cat_gn or conv3x3 or graph_step_bitwise or full_model or graph_train_step or model_hip_vs" > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for e in 1 0; do
  D3D_GNB_EPI=$e timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16_e${e}_$rep.json 2> $O/b16.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b16_e${e}_$rep.json'));print('b16 gnb_epi=$e', d['value'], d['ms_per_step'])"
done; done
for e in 1 0; do
  D3D_GNB_EPI=$e timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_e$e.json 2> $O/b128.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b128_e$e.json'));print('b128 gnb_epi=$e', d['value'], d['ms_per_step'])"
done
