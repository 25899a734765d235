#!/bin/bash
# FWT tests, then cfg4 (FWT-2D) step time with the compile-time-level row kernels (JW_FWT_ROW=1,
# default) against the runtime-level cascades (0), then a kernel-stats profile.  Usage: TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/abrow_$1"; mkdir -p "$O"
cd "$R" || exit 2
timeout -k 10 600 python -u -m pytest tests/test_fwt_gpu.py tests/test_wpt_gpu.py -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  JW_FWT_ROW=$m timeout -k 10 120 python3 bench.py --workload fwt2d --steps 5 --warmup 2 \
    --no-cpu-baseline > "$O/m$m.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "m $m rc=$rc"; tail -5 "$O/m$m.log"; exit $rc; }
  echo "row $m $(grep -h '^{' "$O/m$m.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['roofline']['fwd_ms'], d['roofline']['rev_ms'], d.get('spot_check_vs_oracle'))")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload fwt2d --steps 3 --warmup 1 --no-cpu-baseline --no-check > "$O/prof.log" 2>&1
echo "prof rc=$?"
