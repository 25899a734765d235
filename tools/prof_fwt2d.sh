#!/bin/bash
# FWT 2-D (cfg4) kernel split + FETCH/WRITE per kernel.  Usage: tools/prof_fwt2d.sh TAG [bench args]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-f}"; shift
O="$R/gpurun_out/proffwt_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload fwt2d --steps 2 --warmup 1 --no-cpu-baseline --no-check \
    $BENCH_ARGS > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }
}
run stats --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
