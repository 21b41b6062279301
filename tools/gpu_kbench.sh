# Kernel micro-benchmarks on the X-UNet's real shapes (tools/kbench.py):
#   bash tools/gpu_kbench.sh conv,dgrad,wgrad,linear [--torch]
set -o pipefail
cd /root/repo
O=gpurun_out
OPS=${1:-conv,dgrad,wgrad,linear}
timeout -k 10 900 python tools/kbench.py --ops $OPS --iters 10 --batch 64 ${2:-} > $O/kbench.jsonl 2>$O/kbench.err || exit $?
cat $O/kbench.jsonl
