# round 4: grouped vs per-job weight gradients at the bs128 shapes (isolated), + PMC of the grouped kernel
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python tools/kbench_wgrad_group.py --examples 128 --iters 5 > $O/kb128.jsonl 2> $O/kb.err || exit $?
cut -c1-150 $O/kb128.jsonl
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=/root/repo
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d /root/repo/$O/p1 -o run -- python3 /root/repo/tools/kbench_wgrad_group.py --iters 2 > /root/repo/$O/p1.log 2>&1 || exit $?
python3 /root/repo/tools/pmc_summary.py /root/repo/$O/p1 > /root/repo/$O/summary.txt
head -40 /root/repo/$O/summary.txt
