set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --global_batch 16 > gpurun_out/bench_bs16.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --global_batch 16 --profile gpurun_out/prof_bs16.txt > gpurun_out/bench_bs16_prof.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/rp128 -o run -- python3 /root/repo/bench.py --steps 5 --warmup 2 > /root/repo/gpurun_out/rp128.log 2>&1
rc=$?
echo exit $rc
exit $rc
