#!/bin/bash
# Kernel stats of the STRICT AUTO MODWT path at a Bluestein length (n = 10^6, db4 J=8, 16 signals).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/prof_bs_$1"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- \
  python3 "$R/tools/modwt_time.py" --method auto --arith strict --n 1000000 --batch 16 --reps 2 > "$O/log" 2>&1
echo "rc=$?"; grep '^{' "$O/log" | cut -c1-220
