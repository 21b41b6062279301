set -o pipefail
O=$PWD/gpurun_out/r6_abt; mkdir -p $O
v() { python3 -c "import json,sys;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  for bs in 128 16; do
    st=$([ $bs -ge 128 ] && echo 15 || echo 30)
    timeout -k 10 300 python3 -u bench.py --global_batch $bs --steps $st --warmup 4 > $O/new_b${bs}_$r.json 2> $O/new_b${bs}_$r.err || exit 1
    echo "new b$bs r$r $(v $O/new_b${bs}_$r.json)"
    (cd build/oldtree && timeout -k 10 300 python3 -u bench.py --global_batch $bs --steps $st --warmup 4 > $O/old_b${bs}_$r.json 2> $O/old_b${bs}_$r.err) || exit 1
    echo "old b$bs r$r $(v $O/old_b${bs}_$r.json)"
  done
done
