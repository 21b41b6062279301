set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/rp16 -o run -- python3 /root/repo/bench.py --steps 10 --warmup 2 --global_batch 16 > /root/repo/gpurun_out/rp16.log 2>&1
