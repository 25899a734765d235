#!/bin/bash
# GPU parity tests only (optionally a -k filter), each run under its own time limit.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="${1:-t}"; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 120 \
  --timeout-method thread "$@" > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu_$TAG.log
exit $rc
