#!/bin/bash
# A/B sweep of kernel variants (one bench process per variant, same box).
# Usage: tools/sweep.sh TAG "ENV=v,ENV2=w" "ENV=x" ...   (arith list: SWEEP_ARITH, default fma)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="$1"; shift
OUT="gpurun_out/sweep_$TAG.log"
: > "$OUT"
for arith in ${SWEEP_ARITH:-fma}; do
  for spec in "$@"; do
    env $(echo "$spec" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 6 --warmup 2 \
        --arith $arith --no-cpu-baseline --no-check --no-alt > /tmp/sw.json 2>/dev/null
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $arith $spec rc=$rc" >> "$OUT"; cat "$OUT"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('/tmp/sw.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$arith $spec', d['value'], 'fwd_ms', r['fwd_ms'], 'inv_ms', r['inv_ms'])" >> "$OUT"
  done
done
cat "$OUT"
