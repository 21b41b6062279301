# The perturbed captured step (race-probe snapshot copies, or the bf16 mirror) at small flush batches.
set -o pipefail
O=gpurun_out/${1:-r6_nan8}; mkdir -p $O
run() { local lab=$1; shift; env D3D_GRAPH_COMM=1 D3D_DIAG_BF16_ANY_BATCH=1 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step [23]|after sync' $O/$lab.txt | sed 's/zero-grad params [0-9]*//' | tr '\n' ' ')"; sleep 2; }
for b in 8 16 24 32; do
  run copyonly_$b D3D_WGRAD_DEFER_BATCH=$b D3D_DIAG_PROBE_COPY_ONLY=1
  run bf16_$b D3D_WGRAD_DEFER_BATCH=$b DIAG_NO_PROBE=1 DIAG_PAYLOAD=bf16
done
