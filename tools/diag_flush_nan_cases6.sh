# Does the captured-collective-step problem follow the number of buckets completed per flush?
# (race-probe copy-only perturbation; bucket size varied)
set -o pipefail
O=gpurun_out/${1:-r6_nan9}; mkdir -p $O
run() { local lab=$1; shift; env D3D_GRAPH_COMM=1 D3D_DIAG_BF16_ANY_BATCH=1 D3D_DIAG_PROBE_COPY_ONLY=1 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^defer|^step [23]|after sync' $O/$lab.txt | sed 's/zero-grad params [0-9]*//' | tr '\n' ' ')"; sleep 2; }
run b16_mb2 D3D_WGRAD_DEFER_BATCH=16 DIAG_BUCKET_MB=2
run b16_mb4 D3D_WGRAD_DEFER_BATCH=16 DIAG_BUCKET_MB=4
run b8_mb1 D3D_WGRAD_DEFER_BATCH=8 DIAG_BUCKET_MB=1
run b64_mb64 D3D_WGRAD_DEFER_BATCH=64 DIAG_BUCKET_MB=64
run b64_mb256 D3D_WGRAD_DEFER_BATCH=64 DIAG_BUCKET_MB=256
