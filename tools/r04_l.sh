# round-4 call l: STRICT FFT / AUTO at default three-pass geometry (2^25..2^27); AUTO timing with
# the column kernels' load staging skipped (timing-only build "nostage": values wrong)
mkdir -p gpurun_out/l && timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py -k "default_geometry or auto_2_25" > gpurun_out/l/pytest_long.log 2>&1; rc=$?; tail -8 gpurun_out/l/pytest_long.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/l
for rep in 1 2; do
  for lib in libjwave_hip.so ab/libjwave_hip_nostage.so; do
    JWAVE_HIP_LIB=$PWD/jwave-pro_amd/$lib timeout -k 10 300 python3 tools/modwt_time.py --method auto \
      --arith strict --batch 128 --reps 3 --wavelet Daubechies4 --levels 8 > $O/one.log 2>&1 || { echo "$lib failed"; tail -5 $O/one.log; exit 1; }
    echo "$lib $(tail -1 $O/one.log)" | tee -a $O/nostage.log
  done
done
