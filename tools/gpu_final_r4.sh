#!/bin/bash
# round-4 end-of-round evidence: full GPU suite, smoke, benches (bs128, bs16, bs32, sampling), 128px
set -o pipefail
O=gpurun_out/${FINAL_OUT:-final_r4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench128.json 2> $O/bench128.err || { tail $O/bench128.err; exit 1; }
timeout -k 10 300 python bench.py --global_batch 16 --steps 30 --warmup 5 > $O/bench16.json 2> $O/bench16.err || { tail $O/bench16.err; exit 1; }
timeout -k 10 300 python bench.py --global_batch 32 --steps 20 --warmup 5 > $O/bench32.json 2> $O/bench32.err || { tail $O/bench32.err; exit 1; }
timeout -k 10 400 python bench.py --mode sample > $O/sample.json 2> $O/sample.err || { tail $O/sample.err; exit 1; }
timeout -k 10 400 python bench.py --imgsize 128 --global_batch 16 --steps 10 --warmup 3 > $O/bench128px_16.json 2> $O/b128px.err || { tail $O/b128px.err; exit 1; }
for f in bench128 bench16 bench32 sample bench128px_16; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['unit'],d.get('ms_per_step'))"; done
