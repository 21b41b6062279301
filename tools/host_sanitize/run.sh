# Build the native library's HOST code with AddressSanitizer + UBSan (device
# code uninstrumented: -fsanitize flags go through -Xarch_host) and run the
# planner harness on the CPU.  No GPU needed.
#   bash tools/host_sanitize/run.sh
set -eo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/build/host_sanitize
mkdir -p $OUT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
objs=()
for f in $ROOT/distributed_3d_diffusion_pytorch_amd/ops/csrc/*.hip; do
  o=$OUT/$(basename ${f%.hip}).o
  /opt/rocm/bin/hipcc -std=c++17 -fPIC --offload-arch=gfx950 -O1 -g $SAN -c $f -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $SAN ${objs[@]} -o $OUT/libd3d_hip_asan.so
/opt/rocm/bin/hipcc -std=c++17 -O1 -g $SAN $ROOT/tools/host_sanitize/planners.cpp -L$OUT -ld3d_hip_asan \
  -Wl,-rpath,$OUT -o $OUT/planners
ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1 $OUT/planners
