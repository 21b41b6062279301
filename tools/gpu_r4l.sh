#!/bin/bash
# torch-profiler stacks of the step's remaining at::native kernels (bs128 eager, bs16 eager)
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 300 python bench.py --steps 2 --warmup 2 --profile $O/stack128.txt --profile_stack 10 > $O/b128.json 2> $O/b128.err || { tail $O/b128.err; exit 1; }
timeout -k 10 300 python bench.py --global_batch 16 --graph 0 --steps 2 --warmup 2 --profile $O/stack16.txt --profile_stack 10 > $O/b16.json 2> $O/b16.err || { tail $O/b16.err; exit 1; }
