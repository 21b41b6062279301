set -o pipefail
cd /root/repo
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py --torch --iters 10 > gpurun_out/kbench.jsonl 2> gpurun_out/kbench.err
echo "kbench exit $?"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1
echo "list exit $?"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc1 -- python $R/tools/kbench.py --ops conv --iters 3 > $R/gpurun_out/pmc1.log 2>&1
echo "pmc exit $?"
