#!/bin/bash
# Round-3 evidence: every bench workload (bench_all2.sh), the cwt / fwt2d HBM traffic passes
# (pmc_traffic.sh), and rocprofv3 kernel stats of the headline bench.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r03}"
bash "$R/tools/bench_all2.sh" "$TAG" || exit $?
bash "$R/tools/pmc_traffic.sh" "$TAG" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-check > "$R/gpurun_out/prof_bench_$TAG.log" 2>&1
echo "rocprof rc=$?"
