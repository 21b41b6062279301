# Isolated 64x64-level 128-channel weight gradient at 16 examples per GPU
# (N=32 frames): kernel + split reduction times per wgrad split target.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/wg64
mkdir -p $O
for t in 256 512 1024; do
  D3D_WGRAD_TARGET=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t$t -o run -- python3 /root/repo/tools/conv_one.py --wgrad w8 --n 32 --h 64 --ci 128 --co 128 --iters 20 > $O/t$t.log 2>&1 || exit $?
  db=$(find $O/t$t -name '*.db' | head -n1)
  echo "== target $t"; python3 /root/repo/tools/rpstats.py "$db" --steps 23 --top 6 --grid
  find $O/t$t -name '*.db' -delete
done
