# The flush-batch-64 NaN of the captured 1-rank RCCL step under variations (tools/diag_flush_nan.py).
set -o pipefail
O=gpurun_out/${1:-r6_nan4}; mkdir -p $O
run() { local lab=$1; shift; env D3D_WGRAD_DEFER_BATCH=64 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step [23]|after sync' $O/$lab.txt | sed 's/zero-grad params [0-9]*//' | tr '\n' ' ')"; sleep 2; }
run graph D3D_GRAPH_COMM=1
run graph_noprobe D3D_GRAPH_COMM=1 DIAG_NO_PROBE=1
run graph_noside D3D_GRAPH_COMM=1 D3D_WGRAD_STREAM=0
run graph_nocond D3D_GRAPH_COMM=1 D3D_COND_STREAM=0
run seg D3D_GRAPH_COMM=0 D3D_GRAPH_SEG=64
run graph_bf16 D3D_GRAPH_COMM=1 DIAG_PAYLOAD=bf16
