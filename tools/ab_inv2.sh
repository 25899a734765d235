#!/bin/bash
# Interleaved A/B of the inverse kernels (bench only).  Usage: tools/ab_inv2.sh TAG ORDER... -- [bench args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="$1"; shift
KS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do KS+=("$1"); shift; done
[ "$1" == "--" ] && shift
i=0
for k in "${KS[@]}"; do
  i=$((i+1))
  JW_INV_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${TAG}_$i_$k.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench($k) rc=$rc"; tail -5 gpurun_out/ab_${TAG}_$i_$k.log; exit $rc; fi
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_${TAG}_$i_$k.log') if l.startswith('{')][-1])
r=d['roofline']; o=d.get('other_arith') or {}
print('$i $k', d['value'], d['ms_per_step'], 'fwd', r['fwd_ms'], 'inv', r['inv_ms'], d.get('spot_check_vs_oracle'), 'strict inv', o.get('inv_ms'), o.get('spot_check_vs_oracle'))"
done
