#!/bin/bash
# JW_HOST bounce ring: depth x size at equal or lower pinned memory
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
for rep in 1 2; do for cfg in "4 16" "3 32" "4 32" "4 24" "3 16"; do
  set -- $cfg
  JW_PIN_RING=$1 JW_PIN_MB=$2 timeout -k 10 120 python3 tools/host_time.py > gpurun_out/host_ring.log 2>&1 || { tail -3 gpurun_out/host_ring.log; exit 1; }
  echo "ring=$1 mb=$2 $(grep -o '"ms_per_fwd_inv": [0-9.]*, "msamples_s": [0-9.]*' gpurun_out/host_ring.log)"
done; done
