# bs128 eager (bench default) vs HIP-graph step, same box, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6_g128}; mkdir -p $O
v() { python3 -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])"; }
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --global_batch 128 --steps 15 --warmup 4 > $O/eager_$r.json 2> $O/eager_$r.err || exit 1
  echo "eager r$r $(v $O/eager_$r.json)"
  timeout -k 10 400 python3 -u bench.py --global_batch 128 --steps 15 --warmup 4 --graph 1 > $O/graph_$r.json 2> $O/graph_$r.err || exit 1
  echo "graph r$r $(v $O/graph_$r.json)"
done
