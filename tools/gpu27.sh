set -o pipefail
cd /root/repo
timeout -k 10 600 python tools/kbench.py --ops linear --iters 10 --batch 64 > gpurun_out/kbench_lin.jsonl 2>gpurun_out/kbench.err
