set -o pipefail
cd /root/repo
timeout -k 10 600 python tools/kbench.py --ops conv,dgrad --iters 10 --batch 64 > gpurun_out/kbench_korder.jsonl 2>gpurun_out/kbench_korder.err
