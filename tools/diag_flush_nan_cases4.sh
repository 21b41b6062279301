# Is the probed / bf16 captured-step NaN caused by the separate-buffer collective or by a race its extra
# copy exposes?  (64-job batches)
set -o pipefail
O=gpurun_out/${1:-r6_nan7}; mkdir -p $O
run() { local lab=$1; shift; env D3D_GRAPH_COMM=1 D3D_WGRAD_DEFER_BATCH=64 D3D_DIAG_BF16_ANY_BATCH=1 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 comm > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step [23]|after sync' $O/$lab.txt | sed 's/zero-grad params [0-9]*//' | tr '\n' ' ')"; sleep 2; }
run probe_full
run probe_copyonly D3D_DIAG_PROBE_COPY_ONLY=1
run bf16_noprobe DIAG_NO_PROBE=1 DIAG_PAYLOAD=bf16
run bf16_noprobe_noside DIAG_NO_PROBE=1 DIAG_PAYLOAD=bf16 D3D_WGRAD_STREAM=0
run bf16_noprobe_nodefer DIAG_NO_PROBE=1 DIAG_PAYLOAD=bf16 D3D_DEFER_UPDATE=0
