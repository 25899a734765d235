#!/bin/bash
# Round evidence in one GPU session: full parity suite + headline bench + rocprof stats
# (tools/gpu_check.sh), every bench workload (tools/bench_all2.sh), then the HBM traffic
# passes of the cwt / fwt2d workloads (tools/pmc_traffic.sh).  Stops at the first failure.
# Usage: tools/evidence.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r02}"
bash "$R/tools/gpu_check.sh" "$TAG" || exit $?
bash "$R/tools/bench_all2.sh" "$TAG" || exit $?
bash "$R/tools/pmc_traffic.sh" "$TAG" || exit $?
