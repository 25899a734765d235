#!/bin/bash
# Round-4 check on the GPU box: new boundary tests, the whole GPU suite, the default bench line
# and the row-shape microbenchmark.  Every GPU step under its own limit; stops at the first
# failure.  Usage: tools/r04_check.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-a}"
O=gpurun_out/r04_$TAG
mkdir -p "$O"
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "$O/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_new 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread -k "jni or host_pipeline or cfg3_full or capi or host_threads"
step pytest_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread
step bench 300 python bench.py
[ -x tools/micro/rowshape_bin ] && step rowshape 300 tools/micro/rowshape_bin
exit 0
