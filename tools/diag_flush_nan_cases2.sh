# Production (no race probe) captured 1-rank RCCL step at the flush batches where the probed step fails.
set -o pipefail
O=gpurun_out/${1:-r6_nan5}; mkdir -p $O
run() { local lab=$1; shift; env DIAG_NO_PROBE=1 D3D_GRAPH_COMM=1 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step [23]|after sync' $O/$lab.txt | tr '\n' ' ')"; sleep 2; }
run b48 D3D_WGRAD_DEFER_BATCH=48
run b128 D3D_WGRAD_DEFER_BATCH=128
run b64_bf16 D3D_WGRAD_DEFER_BATCH=64 DIAG_PAYLOAD=bf16
run bflush64 D3D_WGRAD_DEFER_BATCH=64 D3D_WGRAD_BUCKET_FLUSH=1
run bflush64_bf16 D3D_WGRAD_DEFER_BATCH=64 D3D_WGRAD_BUCKET_FLUSH=1 DIAG_PAYLOAD=bf16
run early_b32 D3D_WGRAD_DEFER_BATCH=32 D3D_FILM_EARLY_WGRAD=1
