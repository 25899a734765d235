#!/bin/bash
# A/B of two experimental library builds (jwave-pro_amd/ab/, not part of the product):
#  row40:  FWT row kernels instantiated up to 40 taps (kRowMaxM = 40) -> the FWT/WPT parity tests
#  nt1024: the STRICT FFT column kernels with 1024-thread workgroups -> STRICT parity + timing
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O=gpurun_out/ab_libs; mkdir -p $O
JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_row40.so timeout -k 10 600 python -u -m pytest \
  tests/test_fwt_gpu.py tests/test_wpt_gpu.py -q -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/row40_pytest.log 2>&1
echo "row40 pytest rc=$?"; tail -3 $O/row40_pytest.log
for lib in libjwave_hip.so ab/libjwave_hip_nt1024.so libjwave_hip.so ab/libjwave_hip_nt1024.so; do
  JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 120 python3 tools/modwt_time.py --method auto --arith strict > $O/t.log 2>&1 || { echo "time rc=$?"; tail -3 $O/t.log; exit 1; }
  echo "$lib $(grep '^{' $O/t.log | cut -c1-200)"
done
JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_nt1024.so timeout -k 10 600 python -u -m pytest \
  tests/test_modwt_strict_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/nt1024_pytest.log 2>&1
echo "nt1024 pytest rc=$?"; tail -3 $O/nt1024_pytest.log
