#!/bin/bash
# cfg3 CWT step time against the band cut-off JW_CWT_BAND (max 512-bin blocks per one-pass scale).
# Usage: tools/sweep_band.sh TAG [values...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
O="$R/gpurun_out/sweepband_$TAG"; mkdir -p "$O"
for nb in "$@"; do
  JW_CWT_BAND=$nb timeout -k 10 120 python3 "$R/bench.py" --workload cwt --steps 5 --warmup 2 \
    --no-cpu-baseline --no-check > "$O/nb$nb.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "nb $nb rc=$rc"; tail -5 "$O/nb$nb.log"; exit $rc; }
  echo "nb $nb $(grep -h '^{' "$O/nb$nb.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
done
