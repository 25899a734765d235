#!/bin/bash
# Round-3 final-tree evidence in one call: the whole -m gpu suite, every bench workload
# (bench_all2.sh), the cwt / fwt2d HBM traffic passes and rocprofv3 kernel stats of the
# headline bench.  Each GPU step has its own time limit; a failure ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="${1:-r03c}"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash tools/r03_evidence.sh "$TAG"
