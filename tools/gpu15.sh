set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TA_TA_BUSY GRBM_GUI_ACTIVE --output-format csv -d /root/repo/gpurun_out/pmc2 -o run -- python3 /root/repo/tools/kbench.py --ops conv --iters 2 --batch 64 > /root/repo/gpurun_out/pmc2.log 2>&1
