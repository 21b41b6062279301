# round 4: grouped weight gradients, wide tiles and planner target -- numerics, isolated batches, bs16 A/B
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "wgrad_group or graph_step_bitwise" > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for wide in 1 0; do for blk in 512 1024; do
  D3D_WGRAD_GROUP_WIDE=$wide D3D_WGRAD_GROUP_BLOCKS=$blk timeout -k 10 200 python tools/kbench_wgrad_group.py --blocks $blk > $O/kb_w${wide}_b$blk.jsonl 2> $O/kb.err || exit $?
  echo "wide=$wide blocks=$blk"; cut -c1-160 $O/kb_w${wide}_b$blk.jsonl
done; done
for rep in 1 2; do for cfg in "1 512" "1 1024" "0 512" "0 1024"; do
  set -- $cfg
  D3D_WGRAD_GROUP_WIDE=$1 D3D_WGRAD_GROUP_BLOCKS=$2 timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16_w$1_b$2_$rep.json 2> $O/b16.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b16_w$1_b$2_$rep.json'));print('b16 wide=$1 blocks=$2', d['value'], d['ms_per_step'])"
done; done
