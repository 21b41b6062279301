set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python tools/kbench.py --ops linear --iters 10 --batch 64 --torch > $O/kbench_lin.jsonl 2>$O/kbench_lin.err || exit $?
cut -c1-200 $O/kbench_lin.jsonl
