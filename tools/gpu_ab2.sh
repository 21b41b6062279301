# A/B of the full training step: default kernels vs D3D_FILM_WGRAD=mfma (bs128 and bs16)
set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1; do
timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/ab_new128.json 2>/dev/null || exit $?
D3D_FILM_WGRAD=mfma timeout -k 10 300 python bench.py --steps 15 --warmup 4 > $O/ab_old128.json 2>/dev/null || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/ab_new16.json 2>/dev/null || exit $?
D3D_FILM_WGRAD=mfma timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global_batch 16 > $O/ab_old16.json 2>/dev/null || exit $?
for f in ab_new128 ab_old128 ab_new16 ab_old16; do echo "$f $(cut -c1-170 $O/$f.json)"; done
done
