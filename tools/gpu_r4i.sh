#!/bin/bash
# 128x128: graph-step with the conditioning stream (bs16 = each GPU's share of config 4; bs128 as two
# micro-batches of 64, eager vs graph)
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python bench.py --imgsize 128 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -30 $O/$tag.err; exit 1; }; tail -c 600 $O/$tag.json; echo; }
run g16 --global_batch 16 --steps 10 --warmup 3
D3D_COND_STREAM=0 run g16_nocs --global_batch 16 --steps 10 --warmup 3
run e128 --steps 4 --warmup 2
run g128 --graph 1 --steps 4 --warmup 2
