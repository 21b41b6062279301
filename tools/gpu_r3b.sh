set -o pipefail
O=gpurun_out
mkdir -p $O
DIAG_SERIAL_SIDE=1 DIAG_CONCURRENT=none timeout -k 10 300 python -u tools/diag_determinism.py e:s,e:s,e:sc,e:sc,e:sc,e:sc > $O/diag5_kinds.txt 2>&1 || exit $?
kinds=$(grep "job kinds" $O/diag5_kinds.txt | sed "s/job kinds: //; s/[][',]//g")
echo "kinds: $kinds"
for k in $kinds; do
  DIAG_SERIAL_SIDE=1 DIAG_CONCURRENT=$k timeout -k 10 300 python -u tools/diag_determinism.py e:s,e:s,e:s,e:s,e:s,e:s > $O/diag5_$k.txt 2>&1 || exit $?
  echo "== concurrent kind $k"; grep -v amdgpu.ids $O/diag5_$k.txt | grep "losses equal\|slot hand"
done
grep -v amdgpu.ids $O/diag5_kinds.txt | grep "losses equal\|slot hand"
