#!/bin/bash
# Round-4 profile pass: per-kernel times (rocprofv3 --kernel-trace --stats) and HBM bytes
# (FETCH_SIZE / WRITE_SIZE, separate passes) for JWave's default path (AUTO STRICT, db4 J=8,
# 128 x 2^20), and kernel stats for cfg4 STRICT and cfg5.  Every step under its own limit;
# stops at the first failure.  Usage: tools/prof_r04.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/prof_r04_$1"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # name, limit, rocprof args..., -- is added before the program
  local name=$1 lim=$2; shift 2
  timeout -s KILL "$lim" rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- \
    $PROG > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }
}
PROG="python3 $R/tools/modwt_time.py --method auto --arith strict --batch 128 --reps 2"
timeout -k 10 300 python3 "$R/tools/modwt_time.py" --method auto --arith strict --batch 128 --reps 3 \
  > "$O/auto_time.log" 2>&1 || { echo auto_time failed; tail -5 "$O/auto_time.log"; exit 1; }
tail -1 "$O/auto_time.log"
run auto_stats 300 --kernel-trace --stats
run auto_fetch 300 --kernel-trace --pmc FETCH_SIZE
run auto_write 300 --kernel-trace --pmc WRITE_SIZE
PROG="python3 $R/bench.py --workload fwt2d --arith strict --steps 2 --warmup 1 --no-cpu-baseline --no-check"
run fwt2d_strict_stats 300 --kernel-trace --stats
PROG="python3 $R/bench.py --wavelet Symlet8 --levels 6 --steps 2 --warmup 1 --no-cpu-baseline --no-check --no-alt"
run cfg5_stats 300 --kernel-trace --stats
exit 0
