# round-4 call m: register-I/O column kernels (variant "regio"): STRICT parity, AUTO timing
# against the product; then the STRICT FFT / AUTO tests at the default three-pass geometry
mkdir -p gpurun_out/m
JWAVE_HIP_LIB=$PWD/jwave-pro_amd/ab/libjwave_hip_regio.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py tests/test_fft_gpu.py tests/test_jni_glue_gpu.py -k "not default_geometry and not auto_2_25" > gpurun_out/m/pytest_regio.log 2>&1; rc=$?; tail -3 gpurun_out/m/pytest_regio.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/m
for rep in 1 2; do
  for lib in libjwave_hip.so ab/libjwave_hip_regio.so; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JWAVE_HIP_LIB=$PWD/jwave-pro_amd/$lib timeout -k 10 300 python3 tools/modwt_time.py --method auto \
        --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > $O/one.log 2>&1 || { echo "$lib failed"; tail -5 $O/one.log; exit 1; }
      echo "$lib $wn $(tail -1 $O/one.log)" | tee -a $O/ab.log
    done
  done
done
timeout -k 10 420 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py -k "default_geometry or auto_2_25" > gpurun_out/m/pytest_long.log 2>&1; rc=$?; tail -6 gpurun_out/m/pytest_long.log; exit $rc
