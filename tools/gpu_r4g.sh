# round 4: kernel traces of bs16 / bs128 with and without the GN-backward dgrad-epilogue partials
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=/root/repo/gpurun_out/r4g
mkdir -p $O
for e in 1 0; do
  D3D_GNB_EPI=$e timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db16_$e -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --global_batch 16 > $O/b16_$e.log 2>&1 || exit $?
  db=$(find $O/db16_$e -name '*.db' | head -n1)
  python3 /root/repo/tools/rpstats.py "$db" --window 140 --steps 5 --top 120 --grid > $O/grid16_$e.txt
  python3 /root/repo/tools/rpstats.py "$db" --window 140 --steps 5 --top 80 > $O/stats16_$e.txt
  find $O/db16_$e -name '*.db' -delete
  D3D_GNB_EPI=$e timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db128_$e -o run -- python3 /root/repo/bench.py --steps 8 --warmup 3 > $O/b128_$e.log 2>&1 || exit $?
  db=$(find $O/db128_$e -name '*.db' | head -n1)
  python3 /root/repo/tools/rpstats.py "$db" --window 670 --steps 5 --top 120 --grid > $O/grid128_$e.txt
  python3 /root/repo/tools/rpstats.py "$db" --window 670 --steps 5 --top 80 > $O/stats128_$e.txt
  find $O/db128_$e -name '*.db' -delete
done
for f in grid16_1 grid16_0 grid128_1 grid128_0; do echo "== $f"; grep -E "halo_k<64, true|gn_bwd" $O/$f.txt | head -12; done
for rep in 1 2; do for e in 1 0; do
  D3D_GNB_EPI=$e timeout -k 10 200 python3 /root/repo/bench.py --global_batch 16 --steps 40 --warmup 8 > $O/bb16_e${e}_$rep.json 2> $O/b16.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bb16_e${e}_$rep.json'));print('b16 gnb_epi=$e', d['value'], d['ms_per_step'])"
done; done
for e in 1 0; do
  D3D_GNB_EPI=$e timeout -k 10 300 python3 /root/repo/bench.py --steps 15 --warmup 4 > $O/bb128_e$e.json 2> $O/b128.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bb128_e$e.json'));print('b128 gnb_epi=$e', d['value'], d['ms_per_step'])"
done
