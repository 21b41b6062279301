# Same-box sweep of the in-graph weight-gradient flush policy on the 1-rank RCCL rehearsal of the
# 8-GPU per-GPU step (bs16, captured collectives): job-count batches and work-based (GFLOP) flushing.
#   gpurun -- 'bash tools/defer_batch_sweep.sh <out> "<batch>:<gflop> ..."'
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"
for r in 1 2; do
  for cfg in $2; do
    b=${cfg%%:*}; g=${cfg##*:}
    D3D_WGRAD_DEFER_BATCH=$b D3D_WGRAD_DEFER_GFLOP=$g D3D_GRAPH_COMM=1 D3D_GRAPH_SEG=64 timeout -k 10 300 \
      python3 -u bench.py --force_comm --global_batch "${BS:-16}" --steps 30 --warmup 4 > "$O/fc_${b}_${g}_$r.json" \
      2> "$O/fc_${b}_${g}_$r.err" || exit 1
    echo "fc batch=$b gflop=$g r=$r $(python3 -c "import json;d=json.loads(open('$O/fc_${b}_${g}_$r.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  done
done
