# In-process A/B of two native-library builds (compile-time kernel changes):
#   python tools/build_native.py --rev <REV>     # old sources -> build/ab/<REV>/libd3d_hip.so
#   bash tools/gpu_ab_lib.sh <REV> [bs ...]      # interleaved benches: old (D3D_LIB_PATH) vs the in-tree build
set -o pipefail
cd /root/repo
O=gpurun_out
REV=${1:?rev}; shift
BS=${@:-"16 32 128"}
show() { python3 -c "import json;d=json.load(open('$1'));print(d['value'],d['ms_per_step'])"; }
for round in 1 2; do
  for bs in $BS; do
    st=$([ $bs -ge 128 ] && echo 15 || echo 30)
    D3D_LIB_PATH=build/ab/$REV/libd3d_hip.so timeout -k 10 300 python bench.py --steps $st --warmup 4 --global_batch $bs > $O/abl_old_$bs.json 2>$O/abl_old_$bs.err || exit $?
    echo "bs$bs old($REV) $(show $O/abl_old_$bs.json)"
    timeout -k 10 300 python bench.py --steps $st --warmup 4 --global_batch $bs > $O/abl_new_$bs.json 2>$O/abl_new_$bs.err || exit $?
    echo "bs$bs new       $(show $O/abl_new_$bs.json)"
  done
done
