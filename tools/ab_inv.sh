#!/bin/bash
# A/B of the inverse MODWT kernels on one box: parity tests with the candidate forced, then
# the headline bench with each kernel.  Usage: tools/ab_inv.sh TAG [extra bench args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="${1:-ab}"; shift
JW_INV_KERNEL=wave timeout -k 10 300 python -u -m pytest tests/test_modwt_gpu.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_${TAG}_pytest.log 2>&1
rc=$?; echo "pytest(wave) rc=$rc"; tail -3 gpurun_out/ab_${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for k in wave wg; do
  JW_INV_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_${TAG}_$k.log 2>&1
  rc=$?; echo "bench($k) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${TAG}_$k.log; exit $rc; fi
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_${TAG}_$k.log') if l.startswith('{')][-1])
r=d['roofline']; print('$k', d['value'], d['ms_per_step'], 'fwd', r['fwd_ms'], 'inv', r['inv_ms'], d.get('spot_check_vs_oracle'), d.get('other_arith',{}).get('inv_ms'), d.get('other_arith',{}).get('spot_check_vs_oracle'))"
done
