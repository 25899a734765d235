# round-4 call y: XOR-swizzled LDS columns in JWave's FFT (product) -- STRICT parity, then AUTO
# timing against the 8-point padding (swz0)
mkdir -p gpurun_out/y
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py tests/test_fft_gpu.py tests/test_jni_glue_gpu.py > gpurun_out/y/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/y/pytest.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/y
for rep in 1 2; do
  for lib in libjwave_hip.so ab/libjwave_hip_swz0.so; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JWAVE_HIP_LIB=$PWD/jwave-pro_amd/$lib timeout -k 10 300 python3 tools/modwt_time.py --method auto --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > $O/one.log 2>&1 || { echo "$lib failed"; tail -5 $O/one.log; exit 1; }
      echo "$lib $wn $(tail -1 $O/one.log | cut -c1-220)" | tee -a $O/ab.log
    done
  done
done
