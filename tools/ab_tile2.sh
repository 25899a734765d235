#!/bin/bash
# A/B of the STRICT column kernels' workgroup order: shipped (item-major per tile), tile-fastest,
# tile pairs / quads (P adjacent tiles interleaved, items back to back per group).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O=gpurun_out/ab_tile2; mkdir -p $O
for rep in 1 2; do
for lib in libjwave_hip.so ab/libjwave_hip_tile.so ab/libjwave_hip_tp2.so ab/libjwave_hip_tp4.so; do
  for w in "Daubechies4 8" "Symlet8 6"; do
    set -- $w
    JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 120 python3 tools/modwt_time.py --method auto --arith strict --wavelet $1 --levels $2 > $O/t.log 2>&1 || { echo "time rc=$?"; tail -3 $O/t.log; exit 1; }
    echo "$lib $1 $(grep '^{' $O/t.log | cut -c100-200)"
  done
done
done
