set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/b128.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/b16.json 2>/dev/null || exit $?
for f in b128 b16; do echo "$f $(cut -c1-170 $O/$f.json)"; done
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --global_batch 16 --profile $O/tprof16.txt --profile_stack 4 > /dev/null 2>&1 || exit $?
bash tools/gpu_prof.sh
