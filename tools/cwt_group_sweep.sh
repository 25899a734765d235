#!/bin/bash
# CWT: kernel durations of the sequential two-pass schedule at several workspace sizes
# (does a smaller A window stay in the Infinity Cache?).  Usage: tools/cwt_group_sweep.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-g}"
O="$R/gpurun_out/cwtgrp_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export JW_CWT_PIPE=0
for mb in 16 32 64 128 256; do
  JW_CWT_GROUP_MB=$mb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/g$mb" -o run \
    --output-format csv -- python3 "$R/bench.py" --workload cwt --steps 2 --warmup 1 \
    --no-cpu-baseline --no-check > "$O/g$mb.log" 2>&1 || { echo "g$mb failed"; tail -5 "$O/g$mb.log"; exit 1; }
  echo "g$mb ok"
done
