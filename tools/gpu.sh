#!/bin/bash
# One parameterised driver for every GPU-box job (replaces the per-experiment
# gpu_*.sh scripts).  Run through gpurun from the repo root:
#
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh <out> <step> [<step> ...]'
#
# Results land in gpurun_out/<out>/.  Steps run in order; each GPU step has its
# own time limit and the first failure ends the call (no retries, nothing runs
# on the GPU after a fault / abort / time limit).  Steps:
#
#   tests[:<pytest -k expr>]   GPU suite (or a -k subset), one process, per-test timeout
#   smoke                      __graft_entry__.smoke()
#   bench:<bs>[:<steps>]       bench.py --global_batch <bs> (64x64) -> b<bs>.json
#   bench128px:<bs>            bench.py --imgsize 128 --global_batch <bs>
#   sample                     bench.py --mode sample (256 steps, 64 chains)
#   ab:<variant>:<bs,bs..>     same-box A/B: ablib/<variant>/libd3d_hip.so (D3D_LIB_PATH) vs the
#                              in-tree library, interleaved twice per batch size
#   env:<VAR=val>:<bs,bs..>    same-box A/B of an environment knob against the default
#   prof:<bs>                  rocprofv3 kernel trace of the step + rpstats (stats, grid, busy, gaps,
#                              solo, families)
#   env128px:<VAR=val>:<bs>    the env A/B at 128x128 (bench --imgsize 128)
#   envprof:<VAR=val>:<bs>     the same trace with an environment knob set
#   envfc:<V=x[+V2=y]>:<bs>:<graph|seg>  same-box A/B of knobs on the 1-rank RCCL rehearsal (bench --force_comm)
#   pmc:<bs>                   step-level hardware counters (three --pmc passes) -> table_bs<bs>.txt
#   kbench:<tool.py>[:args]    a tools/ kernel micro-benchmark (args: comma-separated)
#   fc:<bs>:<graph|seg|post>[:<MiB>]  1-rank RCCL rehearsal of the multi-GPU step (bench --force_comm) in one comm
#                              mode (seg: segment size) -> fc_<mode><MiB>_b<bs>.json with its comm record
set -o pipefail
OUT=${1:?usage: gpu.sh <out> <step>...}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/gpurun_out/$OUT
mkdir -p "$O"
cd "$ROOT"
export TMPDIR=/tmp

val() { python3 -c "import json,sys;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'],d.get('unit',''),d.get('ms_per_step'),'fallbacks=',d.get('fallbacks'))"; }
die() { echo "[gpu.sh] step '$1' failed (rc $2)"; [ -f "$3" ] && tail -30 "$3"; exit "$2"; }
steps_for() { [ "$1" -ge 128 ] && echo 15 || echo 30; }

bench() {   # bench <label> <args...>
  local lab=$1; shift
  timeout -k 10 300 python3 -u bench.py "$@" > "$O/$lab.json" 2> "$O/$lab.err" || die "bench $lab" $? "$O/$lab.err"
  echo "$lab $(val "$O/$lab.json")"
}

prof() {    # prof <bs>
  local bs=$1 st w
  st=$([ "$bs" -ge 128 ] && echo 8 || echo 20)
  w=$([ "$bs" -ge 128 ] && echo 670 || echo 140)
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace -d "$O/db$bs" -o run -- python3 "$ROOT/bench.py" \
      --steps "$st" --warmup 3 --global_batch "$bs" > "$O/prof_b$bs.log" 2>&1) || die "prof $bs" $? "$O/prof_b$bs.log"
  local db
  db=$(find "$O/db$bs" -name '*.db' | head -n1)
  python3 tools/rpstats.py "$db" --window "$w" --steps 5 --top 80 > "$O/stats$bs.txt"
  python3 tools/rpstats.py "$db" --window "$w" --steps 5 --top 120 --grid > "$O/grid$bs.txt"
  python3 tools/rpstats.py "$db" --busy "$w" > "$O/busy$bs.txt"
  python3 tools/rpstats.py "$db" --gaps "$w" --top 25 > "$O/gaps$bs.txt"
  python3 tools/rpstats.py "$db" --solo "$w" --top 60 > "$O/solo$bs.txt"
  python3 tools/famsum.py "$O/stats$bs.txt" > "$O/families$bs.txt"
  find "$O/db$bs" -name '*.db' -delete
  tail -n1 "$O/prof_b$bs.log" | cut -c1-160; head -3 "$O/stats$bs.txt"; head -4 "$O/busy$bs.txt"
  head -12 "$O/families$bs.txt"
}

pmc() {     # pmc <bs>
  local bs=$1 d=$O/pmc$1
  mkdir -p "$d"
  local p n=0
  for p in "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" FETCH_SIZE WRITE_SIZE; do
    n=$((n + 1))
    # shellcheck disable=SC2086
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $p --kernel-trace -f csv -d "$d/p$n" -o run -- python3 \
        "$ROOT/bench.py" --steps 2 --warmup 1 --global_batch "$bs" > "$d/p$n.log" 2>&1) || die "pmc $bs pass $n" $? "$d/p$n.log"
  done
  python3 tools/pmc_step_table.py "$d/p1" "$d/p2" "$d/p3" > "$O/table_bs$bs.txt" 2>&1
  find "$d" -name '*.csv' -size +30M -delete
  head -40 "$O/table_bs$bs.txt"
}

for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  echo "[gpu.sh] == $step"
  case $kind in
    tests)
      k=()
      [ -n "$a" ] && k=(-k "$a")
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/pytest_gpu.log" 2>&1 || die tests $? "$O/pytest_gpu.log"
      tail -n 2 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || die smoke $? "$O/smoke.log"
      tail -n 1 "$O/smoke.log" ;;
    bench)
      bench "b$a" --global_batch "$a" --steps "${b:-$(steps_for "$a")}" --warmup 4 ;;
    bench128px)
      bench "b128px_$a" --imgsize 128 --global_batch "$a" --steps 10 --warmup 3 ;;
    sample)
      bench sample --mode sample ;;
    ab)
      lib=ablib/$a/libd3d_hip.so
      [ -f "$lib" ] || die "ab $a (no $lib)" 2
      for r in 1 2; do
        for bs in ${b//,/ }; do
          st=$(steps_for "$bs")
          D3D_LIB_PATH=$lib bench "ab_${a}_b${bs}_$r" --global_batch "$bs" --steps "$st" --warmup 4
          bench "ab_base_b${bs}_$r" --global_batch "$bs" --steps "$st" --warmup 4
        done
      done ;;
    env)
      var=${a%%=*}
      for r in 1 2; do
        for bs in ${b//,/ }; do
          st=$(steps_for "$bs")
          export "${a?}"
          bench "env_${var}_b${bs}_$r" --global_batch "$bs" --steps "$st" --warmup 4
          unset "$var"
          bench "env_base_b${bs}_$r" --global_batch "$bs" --steps "$st" --warmup 4
        done
      done ;;
    env128px)                    # env128px:<VAR=val>:<bs>: the env A/B on the 128x128 config
      var=${a%%=*}
      for r in 1 2; do
        export "${a?}"
        bench "env128_${var}_b${b}_$r" --imgsize 128 --global_batch "$b" --steps 10 --warmup 3
        unset "$var"
        bench "env128_base_b${b}_$r" --imgsize 128 --global_batch "$b" --steps 10 --warmup 3
      done ;;
    fc)                          # fc:<bs>:<graph|seg|post>: 1-rank RCCL rehearsal of the multi-GPU step (bench --force_comm)
      case $b in
        graph) gcm=1; gsg=64 ;;
        seg) gcm=0; gsg=${c:-64} ;;
        post) gcm=0; gsg=0 ;;
        *) die "fc mode $b" 2 ;;
      esac
      D3D_GRAPH_COMM=$gcm D3D_GRAPH_SEG=$gsg bench "fc_${b}${c}_b$a" --force_comm --global_batch "$a" \
        --steps "$(steps_for "$a")" --warmup 4
      python3 -c "import json;d=json.loads(open('$O/fc_${b}${c}_b$a.json').read().strip().splitlines()[-1]);print(d.get('comm'))" ;;
    envfc)                       # envfc:<V=x[+V2=y]>:<bs>:<graph|seg>: fc rehearsal with knobs vs without, interleaved x2
      case $c in graph) gcm=1 ;; seg) gcm=0 ;; *) die "envfc mode $c" 2 ;; esac
      for r in 1 2; do
        (for kv in ${a//+/ }; do export "${kv?}"; done
         D3D_GRAPH_COMM=$gcm D3D_GRAPH_SEG=64 bench "envfc_${c}_b${b}_$r" --force_comm --global_batch "$b" \
           --steps "$(steps_for "$b")" --warmup 4) || exit $?
        D3D_GRAPH_COMM=$gcm D3D_GRAPH_SEG=64 bench "envfc_base_${c}_b${b}_$r" --force_comm --global_batch "$b" \
          --steps "$(steps_for "$b")" --warmup 4
      done ;;
    prof) prof "$a" ;;
    envprof)                     # envprof:<VAR=val>:<bs>: a trace with the knob set (files get a _<VAR> suffix)
      var=${a%%=*}
      export "${a?}"
      prof "$b"
      for f in stats grid busy gaps solo families; do mv "$O/$f$b.txt" "$O/${f}${b}_$var.txt"; done
      unset "$var" ;;
    pmc) pmc "$a" ;;
    kbench)
      args=()
      [ -n "$b" ] && IFS=, read -r -a args <<< "$b"
      timeout -k 10 600 python3 -u "tools/$a" "${args[@]}" > "$O/${a%.py}.txt" 2>&1 || die "kbench $a" $? "$O/${a%.py}.txt"
      tail -n 40 "$O/${a%.py}.txt" ;;
    *) echo "[gpu.sh] unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] all steps done"
