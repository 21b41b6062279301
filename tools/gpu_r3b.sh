set -o pipefail
O=gpurun_out
mkdir -p $O
DIAG_HOLD=1 timeout -k 10 300 python -u tools/diag_determinism.py e:s,e:s,e:s,e:s,e:s,e:s,e:s,e:s > $O/diag8.txt 2>&1 || exit $?
echo HOLD; grep -v amdgpu.ids $O/diag8.txt | grep "losses equal"
