# Per-kernel A/B of two native-library builds at one per-GPU batch: rocprofv3
# kernel traces of the steady-state step with build/ab/<REV> (D3D_LIB_PATH) and
# with the in-tree build; per-kernel ms/step over the last 10 steps.
#   bash tools/gpu_prof_ab.sh <REV> [BS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=/root/repo
O=$R/gpurun_out/profab
mkdir -p $O
REV=${1:?rev}; B=${2:-16}
for arm in old new; do
  if [ $arm = old ]; then export D3D_LIB_PATH=$R/build/ab/$REV/libd3d_hip.so; else unset D3D_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp_$arm -o run -- python3 $R/bench.py --steps 20 --warmup 3 --global_batch $B > $O/b_$arm.json 2> $O/b_$arm.err || exit $?
  db=$(find $O/rp_$arm -name '*.db' | head -n1)
  ms=$(python3 -c "import json;print(json.load(open('$O/b_$arm.json'))['ms_per_step'])")
  W=$(python3 -c "print(10*$ms)")
  python3 $R/tools/rpstats.py "$db" --window $W --steps 10 --top 200 --grid > $O/bs${B}_${arm}_grid.txt
  find $O/rp_$arm -name '*.db' -delete
done
