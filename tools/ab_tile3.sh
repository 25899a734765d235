#!/bin/bash
# A/B of the STRICT column kernels' workgroup order: tile-fastest (shipped) vs item groups of
# 2 / 4 per tile (ab/libjwave_hip_ip{2,4}.so), 16 and 64 signals.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O=gpurun_out/ab_tile3; mkdir -p $O
for rep in 1 2; do
for lib in libjwave_hip.so ab/libjwave_hip_ip2.so ab/libjwave_hip_ip4.so; do
  for w in "Daubechies4 8 16" "Symlet8 6 16" "Daubechies4 8 64"; do
    set -- $w
    JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 120 python3 tools/modwt_time.py --method auto --arith strict --wavelet $1 --levels $2 --batch $3 > $O/t.log 2>&1 || { echo "time rc=$?"; tail -3 $O/t.log; exit 1; }
    echo "$lib $1 B=$3 $(grep '^{' $O/t.log | grep -o '"fwd_ms.*msamples_s": [0-9.]*')"
  done
done
done
