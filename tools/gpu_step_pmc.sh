# Hardware counters per kernel of the bs128 training step: three --pmc passes
# (SQ+GRBM / FETCH_SIZE / WRITE_SIZE, each within one pass's counter limits)
# over bench.py, summarised by tools/pmc_step_table.py.   B=16 for the bs16 step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/spmc${B:-128}
mkdir -p $O
B_ARGS=""
[ -n "$B" ] && B_ARGS="--global_batch $B"
run() {
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -f csv -d $O/$P -o run -- python3 /root/repo/bench.py --steps 2 --warmup 1 $B_ARGS > $O/$P.log 2>&1
}
P=p1 run SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || { tail -5 $O/p1.log; exit 1; }
P=p2 run FETCH_SIZE || { tail -5 $O/p2.log; exit 1; }
P=p3 run WRITE_SIZE || { tail -5 $O/p3.log; exit 1; }
python3 /root/repo/tools/pmc_step_table.py $O/p1 $O/p2 $O/p3 > $O/table.txt 2>&1
find $O -name '*.csv' -size +30M -delete
cat $O/table.txt
