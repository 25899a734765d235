#!/bin/bash
# Every bench workload once (each under its own time limit; stops at the first failure).
# Usage: tools/bench_all.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r01}"
mkdir -p gpurun_out
O="gpurun_out/bench_all_$TAG.jsonl"
: > "$O"
run() { timeout -k 10 600 python bench.py "$@" > gpurun_out/ba.log 2>&1 || { tail -5 gpurun_out/ba.log; exit 1; }; grep '^{' gpurun_out/ba.log >> "$O"; }
run
run --wavelet Symlet8 --levels 6 --no-cpu-baseline --no-alt
run --wavelet Symlet8 --levels 6 --global-batch 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-alt
run --workload cwt --steps 3 --warmup 1
run --workload fwt2d --steps 3 --warmup 1
run --workload fwt2d --steps 3 --warmup 1 --arith strict --no-cpu-baseline
echo "wrote $O"
