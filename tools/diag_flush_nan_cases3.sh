# bf16-payload captured-step NaN (64-job batches, no race probe): which streams / features it needs.
set -o pipefail
O=gpurun_out/${1:-r6_nan6}; mkdir -p $O
run() { local lab=$1; shift; env DIAG_NO_PROBE=1 DIAG_PAYLOAD=bf16 D3D_GRAPH_COMM=1 D3D_WGRAD_DEFER_BATCH=64 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 bf16 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step [23]|after sync' $O/$lab.txt | tr '\n' ' ')"; sleep 2; }
run base
run nodefer D3D_DEFER_UPDATE=0
run nocond D3D_COND_STREAM=0
run noside D3D_WGRAD_STREAM=0
run nogroup D3D_WGRAD_GROUP=0
