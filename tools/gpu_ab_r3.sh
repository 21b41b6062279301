# interleaved in-process A/B of the round-3 switches (tools/ab_run.py): bs16 and bs128
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
run() {  # name, env, args
  local name=$1; shift
  local envs=$1; shift
  env $envs timeout -k 10 300 python tools/ab_run.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  for v in "old AB_FILM_EV=0 AB_S64=1" "ev AB_FILM_EV=1 AB_S64=1" "s64 AB_FILM_EV=0 AB_S64=0" "both AB_FILM_EV=1 AB_S64=0"; do
    set -- $v
    n=$1; shift
    run b16_${n}_$r "$*" --global_batch 16 --steps 40 --warmup 8 || exit 1
  done
done
for r in 1 2; do
  for v in "old AB_FILM_EV=0" "ev AB_FILM_EV=1"; do
    set -- $v
    n=$1; shift
    run b128_${n}_$r "$*" --steps 15 --warmup 4 || exit 1
  done
done
