set -o pipefail
O=gpurun_out/r6_nan2; mkdir -p $O
run() { local lab=$1; shift; env D3D_GRAPH_COMM=1 D3D_WGRAD_DEFER_BATCH=32 "$@" timeout -k 10 240 python3 -u tools/diag_flush_nan.py 1 fp32 > $O/$lab.txt 2>&1 || echo "$lab rc=$?"; echo "$lab: $(grep -E '^step 2|after sync' $O/$lab.txt | tr '\n' ' ')"; }
run base
run early0 D3D_FILM_EARLY_WGRAD=0
run wide_off D3D_ATTN_WIDE_MIN=1073741824 D3D_ATTN_FWD_ALL_MIN=1073741824
run defer0 D3D_DEFER_UPDATE=0
run cond1 D3D_COND_STREAM=0
run nostream D3D_WGRAD_STREAM=0
