#!/bin/bash
# A/B of experimental library builds (jwave-pro_amd/ab/libjwave_hip_NAME.so) on JWave's default
# path (AUTO STRICT, 128 x 2^20, db4 J=8 and sym8 J=6), alternating with the product library,
# then the STRICT parity tests on each variant.  Usage: tools/ab_auto_libs.sh TAG NAME [NAME ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O="gpurun_out/ab_auto_libs_$1"; shift; mkdir -p "$O"
LIBS=("libjwave_hip.so")
for n in "$@"; do LIBS+=("ab/libjwave_hip_$n.so"); done
for rep in 1 2; do
  for lib in "${LIBS[@]}"; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 300 python3 tools/modwt_time.py --method auto \
        --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > "$O/one.log" 2>&1 \
        || { echo "$lib failed"; tail -5 "$O/one.log"; exit 1; }
      echo "$lib $(tail -1 "$O/one.log")" | tee -a "$O/ab.log"
    done
  done
done
for n in "$@"; do
  JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_$n.so timeout -k 10 600 python -u -m pytest \
    tests/test_modwt_strict_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_$n.log" 2>&1
  rc=$?; echo "$n pytest rc=$rc"; tail -2 "$O/pytest_$n.log"; [ $rc -eq 0 ] || exit $rc
done
