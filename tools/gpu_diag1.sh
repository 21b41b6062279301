set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 300 python tools/diag_graph.py --batch 16 --mb 16 --steps 5 > $O/diag_graph16.log 2>&1 || exit $?
cat $O/diag_graph16.log
timeout -k 10 300 python tools/diag_graph.py --batch 128 --mb 64 --steps 5 > $O/diag_graph128.log 2>&1 || exit $?
cat $O/diag_graph128.log
timeout -k 10 300 python tools/diag_graph.py --batch 128 --mb 64 --steps 5 --dropout 0 > $O/diag_graph128d0.log 2>&1 || exit $?
cat $O/diag_graph128d0.log
bash tools/gpu_prof.sh
