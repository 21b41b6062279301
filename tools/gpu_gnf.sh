set -o pipefail
cd /root/repo
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_gn or conv3x3 or group_norm or gn_film" > $O/test_gnf.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $O/test_gnf.log | tail -15; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_step.sh
