#!/bin/bash
# A/B of env knobs on cfg3 (CWT Morlet, 64 scales, N=2^18, x256), alternating.
# Usage: tools/ab_cwt.sh TAG "ENV=VAL ..." [...]   (the baseline "" runs first)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O="gpurun_out/ab_cwt_$1"; shift; mkdir -p "$O"
CFGS=("" "$@")
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    env $cfg timeout -k 10 300 python3 bench.py --workload cwt --steps 3 --warmup 1 \
      --no-cpu-baseline --no-check > "$O/one.log" 2>&1 || { echo "[$cfg] failed"; tail -5 "$O/one.log"; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('$O/one.log') if l.startswith('{')][-1])
print('[$cfg]', d['value'], d['ms_per_step'], d['roofline']['frac'])" | tee -a "$O/ab.log"
  done
done
