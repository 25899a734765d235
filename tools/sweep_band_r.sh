#!/bin/bash
# cfg3 CWT step time against JW_CWT_BAND_R (row groups per band workgroup) and the cut-off.
# Usage: tools/sweep_band_r.sh TAG "R values" "nb values"
R0="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R0/gpurun_out/sweepbandr_$1"; mkdir -p "$O"
for r in $2; do for nb in $3; do
  JW_CWT_BAND_R=$r JW_CWT_BAND=$nb timeout -k 10 120 python3 "$R0/bench.py" --workload cwt --steps 5 \
    --warmup 2 --no-cpu-baseline --no-check > "$O/r${r}nb$nb.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "r $r nb $nb rc=$rc"; tail -5 "$O/r${r}nb$nb.log"; exit $rc; }
  echo "R $r nb $nb $(grep -h '^{' "$O/r${r}nb$nb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
done; done
