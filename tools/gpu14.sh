cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > /root/repo/gpurun_out/counters_list.txt 2>&1
echo done
