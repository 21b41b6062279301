#!/bin/bash
# Wave-cycle breakdown of the dense GEMM vs hipBLASLt on one kbench shape:
#   bash tools/pmc_gemm.sh <out> "<kbench --only substring>"
# Two --pmc passes (8 SQ counters max per pass), each under its own time limit.
set -o pipefail
OUT=${1:?out}; ONLY=${2:?shape}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/gpurun_out/$OUT
mkdir -p "$O"
export TMPDIR=/tmp
n=0
for p in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  n=$((n + 1))
  # shellcheck disable=SC2086
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $p --kernel-trace -f csv -d "$O/p$n" -o run -- python3 \
      "$ROOT/tools/kbench_gemm.py" --only "$ONLY" --rounds 1 --iters 3 > "$O/p$n.log" 2>&1) || { echo "pass $n failed"; tail -20 "$O/p$n.log"; exit 1; }
  f=$(find "$O/p$n" -name '*counter_collection.csv' | head -n1)
  python3 "$ROOT/tools/pmcstats.py" "$f" > "$O/stats_p$n.txt"
  head -20 "$O/stats_p$n.txt"
done
find "$O" -name '*.csv' -size +20M -delete
