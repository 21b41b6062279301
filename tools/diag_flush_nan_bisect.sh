# Which weight-gradient flush batches leave non-finite gradients in the captured 1-rank RCCL step
# (and, "nocomm", in the captured single-GPU step): tools/diag_flush_nan.py per batch size.
set -o pipefail
O=gpurun_out/${1:-r6_nan3}; mkdir -p $O
for mode in comm nocomm; do
  for b in ${BATCHES:-8 16 24 32 48 64 96 128}; do
    env D3D_GRAPH_COMM=1 D3D_WGRAD_DEFER_BATCH=$b timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 $mode \
      > $O/${mode}_$b.txt 2>&1 || echo "$mode $b rc=$?"
    echo "$mode b=$b: $(grep -cE 'nonfinite-grad params [1-9]|loss nan' $O/${mode}_$b.txt) bad steps; $(grep -E 'after sync' $O/${mode}_$b.txt)"
  done
done
