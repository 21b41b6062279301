set -o pipefail
cd /root/repo
mkdir -p gpurun_out
(rocm-smi --showproductname --showmeminfo vram || true) > gpurun_out/smi.txt 2>&1
python -c "import distributed_3d_diffusion_pytorch_amd as d; print('import ok', d.__file__)" > gpurun_out/import.txt 2>&1
export D3D_BACKEND=torch MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --global_batch 16 > gpurun_out/bench_torch_bs16.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --micro_batch 32 --profile gpurun_out/prof_torch_bs128.txt > gpurun_out/bench_torch_bs128.log 2>&1
echo exit $?
