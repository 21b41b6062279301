set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d /root/repo/gpurun_out/pmc3 -o run -- python3 /root/repo/tools/kbench.py --ops wgrad --iters 2 --batch 64 > /root/repo/gpurun_out/pmc3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d /root/repo/gpurun_out/pmc4 -o run -- python3 /root/repo/tools/kbench.py --ops wgrad --iters 2 --batch 64 > /root/repo/gpurun_out/pmc4.log 2>&1
