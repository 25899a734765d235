#!/bin/bash
# A/B sweep of kernel variants (one process per variant, same box).  Usage: tools/sweep.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="$1"; shift
OUT="gpurun_out/sweep_$TAG.log"
: > "$OUT"
for arith in fma strict; do
  for ic in 256 384 d3; do
    JW_INV_C=${ic/d3/256} JW_INV_D=$([ $ic = d3 ] && echo 3 || echo 2) timeout -k 10 300 python bench.py --steps 6 --warmup 2 \
        --arith $arith --no-cpu-baseline --no-check "$@" > /tmp/sw.json 2>/dev/null
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $arith $ic rc=$rc" >> "$OUT"; cat "$OUT"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('/tmp/sw.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$arith inv_c=$ic', d['value'], 'fwd_ms', r['fwd_ms'], 'inv_ms', r['inv_ms'])" >> "$OUT"
  done
done
cat "$OUT"
