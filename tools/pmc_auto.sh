#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) over the STRICT AUTO MODWT path at 16 x 2^20
# (tools/modwt_time.py): per-kernel HBM bytes of JWave's default path.  Usage: TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmcauto_$1"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$O/$c" -o run --output-format csv -- \
    python3 "$R/tools/modwt_time.py" --method auto --arith strict --reps 1 > "$O/$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$c.log"; exit $rc; }
done
