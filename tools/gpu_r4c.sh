# round 4: grouped weight gradients with an NS-stage ring and asm transposed reads
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 200 --timeout-method thread \
  -k "wgrad_group or graph_step_bitwise" > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for ns in 2 3 4; do for blk in 512 1024; do
  D3D_WGRAD_GROUP_NS=$ns timeout -k 10 200 python tools/kbench_wgrad_group.py --blocks $blk > $O/kb_ns${ns}_b$blk.jsonl 2> $O/kb.err || exit $?
  echo "ns=$ns blocks=$blk"; cut -c1-130 $O/kb_ns${ns}_b$blk.jsonl
done; done
for rep in 1 2; do for cfg in "4 512" "4 1024" "2 512" "3 512"; do
  set -- $cfg
  D3D_WGRAD_GROUP_NS=$1 D3D_WGRAD_GROUP_BLOCKS=$2 timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/b16_ns$1_b$2_$rep.json 2> $O/b16.err || exit $?
  python3 -c "import json;d=json.load(open('$O/b16_ns$1_b$2_$rep.json'));print('b16 ns=$1 blocks=$2', d['value'], d['ms_per_step'])"
done; done
