set -o pipefail
cd /root/repo
timeout -k 10 600 python bench.py --mode sample > gpurun_out/bench_sample.log 2>&1 || exit 1
tail -n1 gpurun_out/bench_sample.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/rp128 -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 > /root/repo/gpurun_out/rp128.log 2>&1
