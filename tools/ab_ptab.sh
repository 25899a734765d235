#!/bin/bash
# FWT / WPT / CWT parity tests, cfg4 in both arithmetic contracts, then cfg3 (CWT) with the
# two-pass scales' psi_hat tabulated per call (JW_CWT_PTAB=1, default) against per-element
# evaluation (0), twice each, and a kernel-stats profile of cfg4.  Usage: TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/abptab_$1"; mkdir -p "$O"
cd "$R" || exit 2
timeout -k 10 600 python -u -m pytest tests/test_fwt_gpu.py tests/test_wpt_gpu.py tests/test_cwt_gpu.py \
  -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
summ() { grep -h '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], d['value'], r.get('fwd_ms'), r.get('rev_ms'), r['frac'], d.get('spot_check_vs_oracle'), d.get('parity'))"; }
for a in fma strict; do
  timeout -k 10 120 python3 bench.py --workload fwt2d --steps 5 --warmup 2 --arith $a --no-cpu-baseline > "$O/f_$a.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "fwt2d $a rc=$rc"; tail -5 "$O/f_$a.log"; exit $rc; }
  echo "fwt2d $a $(summ "$O/f_$a.log")"
done
for m in 0 1 0 1; do
  JW_CWT_PTAB=$m timeout -k 10 120 python3 bench.py --workload cwt --steps 3 --warmup 1 --no-cpu-baseline > "$O/c$m.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "cwt $m rc=$rc"; tail -5 "$O/c$m.log"; exit $rc; }
  echo "cwt ptab=$m $(summ "$O/c$m.log")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --workload fwt2d --steps 3 --warmup 1 --no-cpu-baseline --no-check > "$O/prof.log" 2>&1
echo "prof rc=$?"
