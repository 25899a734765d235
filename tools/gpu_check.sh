#!/bin/bash
# One GPU session: parity tests, then (only if no crash) the bench and a rocprofv3 kernel trace
# of the headline launches only (--no-check --no-alt --no-cpu-baseline: no host-path, AUTO or
# STRICT legs, so each kernel's average in the stats is the timed launch's duration).
# Every GPU step has its own time limit; a crash/timeout ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="${1:-r01}"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --no-check --no-alt --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 "$R/gpurun_out/prof_$TAG.log"
exit $rc
