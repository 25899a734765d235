#!/bin/bash
# CWT kernel split: rocprofv3 kernel stats with the pipelined and the sequential group schedule,
# then FETCH_SIZE / WRITE_SIZE passes (sequential schedule, so each pass kernel is separate).
# Usage: tools/prof_cwt.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-cwt}"; shift
O="$R/gpurun_out/profcwt_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {  # name, then rocprof args
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$O/$name" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload cwt --steps 2 --warmup 1 --no-cpu-baseline --no-check \
    $BENCH_ARGS > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }
}
run pipe --kernel-trace --stats
export JW_CWT_PIPE=0
run seq --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
