#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel trace only) over the cwt and fwt2d bench
# workloads at their defaults; tools/traffic_summary.py turns them into profiles/ traffic.
# Usage: tools/pmc_traffic.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-t}"
O="$R/gpurun_out/pmctraffic_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for w in cwt fwt2d; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$O/${w}_$c" -o run --output-format csv -- \
      python3 "$R/bench.py" --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-check \
      > "$O/${w}_$c.log" 2>&1
    rc=$?; echo "$w $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/${w}_$c.log"; exit $rc; }
  done
done
