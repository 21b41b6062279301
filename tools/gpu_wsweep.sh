# bufl weight-gradient split-plan sweep (block target x rounding)
set -o pipefail
cd /root/repo
O=gpurun_out
for cfg in "384 0" "512 0" "768 0" "1024 0"; do
  set -- $cfg
  D3D_WGRAD_IMPL=bufl D3D_WGRAD_TARGET=$1 D3D_WGRAD_CEIL=$2 timeout -k 10 300 python tools/kbench.py --ops wgrad --iters 10 --batch 16 > $O/ws.jsonl 2>/dev/null || exit $?
  echo "== target $1 ceil $2"; grep '"hip-bufl"' $O/ws.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
  r=json.loads(l); print(r['shape'], r['us'])"
done
