#!/bin/bash
# Round-4 evidence on one box: the whole GPU suite, smoke(), every bench workload, the cwt / fwt2d
# HBM traffic passes, and rocprofv3 kernel stats of the headline bench.  Stops at a failure.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r04}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash "$R/tools/bench_all2.sh" "$TAG" || exit $?
bash "$R/tools/pmc_traffic.sh" "$TAG" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-check > "$R/gpurun_out/prof_bench_$TAG.log" 2>&1
echo "rocprof rc=$?"
