# bs16 (8-GPU per-GPU share) graph step under HIP runtime settings that govern
# how far the host can enqueue ahead of the device (interleaved, 2 rounds)
set -o pipefail
O=gpurun_out/envab
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --global_batch 16 --steps 40 --warmup 8 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 0; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run base$r X=1
  run aql64k$r ROC_AQL_QUEUE_SIZE=65536
  run pktcap1_$r DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  run pktcap0_$r DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  run hwq8_$r GPU_MAX_HW_QUEUES=8
done
