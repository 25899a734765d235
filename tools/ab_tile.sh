#!/bin/bash
# A/B: STRICT AUTO path with the shipped workgroup order vs tile-fastest order
# (jwave-pro_amd/ab/libjwave_hip_tile.so), timing + FETCH/WRITE of each.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O=gpurun_out/ab_tile; mkdir -p $O
for lib in libjwave_hip.so ab/libjwave_hip_tile.so libjwave_hip.so ab/libjwave_hip_tile.so; do
  JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 120 python3 tools/modwt_time.py --method auto --arith strict > $O/t.log 2>&1 || { echo "time rc=$?"; tail -3 $O/t.log; exit 1; }
  echo "$lib $(grep '^{' $O/t.log | cut -c100-200)"
done
bash tools/pmc_auto.sh base || exit 1
JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_tile.so bash tools/pmc_auto.sh tile || exit 1
JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_tile.so timeout -k 10 600 python -u -m pytest \
  tests/test_modwt_strict_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $O/tile_pytest.log 2>&1
echo "tile pytest rc=$?"; tail -2 $O/tile_pytest.log
