#!/bin/bash
# piecebench timings, then its FETCH_SIZE / WRITE_SIZE per kernel (separate passes)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out/piece_$1"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 "$R/tools/micro/piecebench_bin" > "$O/time.log" 2>&1 || { tail -3 "$O/time.log"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c -d "$O/$c" -o run --output-format csv -- \
    "$R/tools/micro/piecebench_bin" > "$O/$c.log" 2>&1 || { echo "$c failed"; tail -3 "$O/$c.log"; exit 1; }
done
echo done
