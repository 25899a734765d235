#!/bin/bash
# Every bench workload once, each under its own time limit; stops at the first failure.
# Usage: tools/bench_all2.sh TAG  (writes gpurun_out/bench_all_TAG.jsonl)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r02}"
mkdir -p gpurun_out
O="gpurun_out/bench_all_$TAG.jsonl"
: > "$O"
run() { timeout -k 10 600 python bench.py "$@" > gpurun_out/ba_$TAG.log 2>&1 || { tail -5 gpurun_out/ba_$TAG.log; exit 1; }; grep '^{' gpurun_out/ba_$TAG.log >> "$O"; echo "ok: $*"; }
run --workload fwt2d --steps 5 --warmup 2
run --workload fwt2d --steps 5 --warmup 2 --arith strict --no-cpu-baseline
run --workload cwt --steps 3 --warmup 1
run --wavelet Symlet8 --levels 6 --no-cpu-baseline --no-alt
run --wavelet Symlet8 --levels 6 --global-batch 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-alt
run
echo "wrote $O"
