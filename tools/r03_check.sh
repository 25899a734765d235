#!/bin/bash
# Round-3 GPU session: the whole -m gpu suite, the default bench line, and kernel stats of the
# STRICT AUTO MODWT path (JWave's default) at cfg2 geometry.  Each GPU step has its own time
# limit; a crash or timeout ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="${1:-r03}"
SKIP_TESTS="${SKIP_TESTS:-0}"
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python tools/modwt_time.py --method auto --arith strict > gpurun_out/auto_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/modwt_time.py --method auto --arith strict --wavelet Symlet8 --levels 6 >> gpurun_out/auto_$TAG.log 2>&1 &&
timeout -k 10 300 python tools/modwt_time.py --method fft --arith fma >> gpurun_out/auto_$TAG.log 2>&1
rc=$?
echo "modwt_time rc=$rc"; cat gpurun_out/auto_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_auto_$TAG" -o run --output-format csv \
  -- python3 "$R/tools/modwt_time.py" --method auto --arith strict --reps 2 > "$R/gpurun_out/prof_auto_$TAG.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
cd "$R"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$TAG.log
exit $rc
