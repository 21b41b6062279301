# tune the library GEMMs of the one-micro-batch bs128 step (new shapes appended to a copy of the table), then A/B
set -o pipefail
cd /root/repo
O=gpurun_out/tune
mkdir -p $O
cp tuning/tunableop_mi355x.csv $O/tun.csv
D3D_TUNE_MS=30 timeout -k 10 900 python tools/tune_gemms.py --batches 128 --out $O/tun.csv > $O/tune.log 2>&1 || exit $?
grep "\[tune\]" $O/tune.log; wc -l $O/tun.csv
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/old.json 2> $O/old.err || exit $?
  echo "b128 old-table $(show $O/old.json)"
  D3D_TUNED_GEMMS_TABLE=$O/tun.csv timeout -k 10 300 python bench.py --steps 12 --warmup 4 > $O/new.json 2> $O/new.err || exit $?
  echo "b128 new-table $(show $O/new.json)"
done
