# round 4: grouped weight gradients -- numerics, isolated batches, in-step A/B at bs16
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "conv3x3 or wgrad_group or graph_step_bitwise or wgrad_tn or cond_conv or diff_loss or captured_collectives_one_rank or film_batch or graph_train_step or adam or fused_update" > $O/pytest.log 2>&1
rc=$?; tail -n 4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for ra in 1 0; do
  D3D_CONV_RES_ALWAYS=$ra timeout -k 10 200 python tools/kbench_conv_levels.py 32 256 > $O/kconv_ra$ra.jsonl 2> $O/kconv.err || exit $?
  cat $O/kconv_ra$ra.jsonl
done
for pk in 32 64; do
  timeout -k 10 200 python tools/kbench_wgrad_group.py --pk $pk > $O/kb_pk$pk.jsonl 2> $O/kb.err || exit $?
  cat $O/kb_pk$pk.jsonl
done
for g in 1 0 1 0; do
  D3D_WGRAD_GROUP=$g timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16_g$g.json 2> $O/b16.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b16_g$g.json'));print('b16 group=$g', d['value'], d['ms_per_step'])"
done
for g in 0 1; do
  D3D_WGRAD_EAGER_GROUP=$g timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128_e$g.json 2> $O/b128.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b128_e$g.json'));print('b128 eager_group=$g', d['value'], d['ms_per_step'])"
done
