# round-4 call n: register-I/O column kernels with the 8-point LDS padding (regio8) and the
# padding alone (pad8): STRICT parity of regio8, AUTO timing against the product
mkdir -p gpurun_out/n
JWAVE_HIP_LIB=$PWD/jwave-pro_amd/ab/libjwave_hip_regio8.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py tests/test_fft_gpu.py -k "not default_geometry and not auto_2_25" > gpurun_out/n/pytest_regio8.log 2>&1; rc=$?; tail -2 gpurun_out/n/pytest_regio8.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/n
for rep in 1 2; do
  for lib in libjwave_hip.so ab/libjwave_hip_regio8.so ab/libjwave_hip_pad8.so; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JWAVE_HIP_LIB=$PWD/jwave-pro_amd/$lib timeout -k 10 300 python3 tools/modwt_time.py --method auto \
        --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > $O/one.log 2>&1 || { echo "$lib failed"; tail -5 $O/one.log; exit 1; }
      echo "$lib $wn $(tail -1 $O/one.log | cut -c1-200)" | tee -a $O/ab.log
    done
  done
done
