# conditioning stream in the other regimes: 64x64 bs128 as 2 micro-batches, bs64 (the 2-GPU share), 128x128 as one
# micro-batch; ex/s ms/step HBM-GiB
set -o pipefail
cd /root/repo
O=gpurun_out/csr
mkdir -p $O
run() { lab=$1; shift; env $E timeout -k 10 300 python bench.py "$@" > $O/$lab.json 2> $O/$lab.err || exit $?; python3 -c "import json;d=json.load(open('$O/$lab.json'));print('$lab',d['value'],d['ms_per_step'],d['hbm_peak_gib'])"; }
for v in 1 0; do
  E="D3D_COND_STREAM=$v"; run mb64_cs$v --steps 10 --warmup 3 --micro_batch 64
  E="D3D_COND_STREAM=$v"; run bs64_cs$v --steps 15 --warmup 4 --global_batch 64
done
E="X=1"; run px128_mb128 --steps 4 --warmup 2 --imgsize 128 --micro_batch 128
E="X=1"; run px128_mb64 --steps 4 --warmup 2 --imgsize 128
