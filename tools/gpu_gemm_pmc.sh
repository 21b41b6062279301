# PMC passes over the GEMM kernel versions VERS (kbench_gemm.py --vers) and hipBLASLt on one shape:
# wave-state split, MFMA busy, LDS conflicts, effective clock.   SHAPE=sq8192 VERS=3 bash tools/gpu_gemm_pmc.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/${TAG:-pmc}
mkdir -p $O
export PYTHONPATH=/root/repo
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 /root/repo/tools/kbench_gemm.py --only "${SHAPE:-sq8192}" --vers ${VERS:-3} --rounds 1 --iters 5 > $O/p1.log 2>&1 || exit $?
python3 /root/repo/tools/pmc_summary.py $O/p1 > $O/summary.txt
cat $O/summary.txt
