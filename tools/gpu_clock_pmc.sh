# GRBM_GUI_ACTIVE cycles per ns of the heaviest kernels: sustained training step vs short isolated bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/clk
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/step -o run -- python3 /root/repo/bench.py --steps 3 --warmup 2 > $O/step.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/iso -o run -- python3 /root/repo/tools/kbench_conv_epi_r3.py 256 > $O/iso.log 2>&1 || exit $?
python3 /root/repo/tools/pmc_clock.py $O/step > $O/clock_step.txt 2>&1
python3 /root/repo/tools/pmc_clock.py $O/iso > $O/clock_iso.txt 2>&1
find $O -name '*.csv' -size +20M -delete
cat $O/clock_step.txt; echo ---; cat $O/clock_iso.txt
# training sanity: 400 replayed bs16 steps on synthetic SRN-shaped data (loss must fall, stay finite)
cd /root/repo
timeout -k 10 300 python train.py --synthetic --steps 400 --preset cars64_1gpu_bf16 --out_dir gpurun_out/clk/run graph=true log_every=50 ckpt_every=0 optim.warmup_examples=1600 > gpurun_out/clk/train.log 2>&1 || { tail -5 gpurun_out/clk/train.log; exit 1; }
grep -i "loss" gpurun_out/clk/train.log | tail -10
find gpurun_out/clk/run -name '*.pt' -delete
