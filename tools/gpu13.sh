set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d /root/repo/gpurun_out/pmc1 -o run -- python3 /root/repo/tools/kbench.py --ops conv,dgrad,wgrad --iters 3 --batch 64 > /root/repo/gpurun_out/pmc1.log 2>&1
