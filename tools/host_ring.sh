#!/bin/bash
# JW_HOST bounce-ring depth A/B (JW_PIN_RING 2 / 3 / 4) with tools/host_time.py, plus the
# 8-thread host test.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
for rep in 1 2; do for r in 2 3 4; do
  JW_PIN_RING=$r timeout -k 10 120 python3 tools/host_time.py > gpurun_out/host_ring.log 2>&1 || { tail -3 gpurun_out/host_ring.log; exit 1; }
  echo "ring=$r $(grep '^{' gpurun_out/host_ring.log)"
done; done
timeout -k 10 300 python -u -m pytest tests/test_host_threads_gpu.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/host_threads.log 2>&1
echo "host threads rc=$?"; tail -2 gpurun_out/host_threads.log
