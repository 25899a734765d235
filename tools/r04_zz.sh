# round-4 call zz: the product with 512-point FFT columns padded (swizzle from 1024 up):
# STRICT / FFT / JNI GPU tests, AUTO timing, smoke and the default bench
mkdir -p gpurun_out/zz
timeout -k 10 600 python -u -m pytest tests/test_modwt_strict_gpu.py tests/test_fft_gpu.py tests/test_jni_glue_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/zz/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/zz/pytest.log; [ $rc -eq 0 ] || exit $rc
for w in "Daubechies4 8" "Symlet8 6"; do read -r wn wl <<< "$w"
  timeout -k 10 300 python3 tools/modwt_time.py --method auto --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > gpurun_out/zz/one.log 2>&1 || { tail -5 gpurun_out/zz/one.log; exit 1; }
  tail -1 gpurun_out/zz/one.log | tee -a gpurun_out/zz/auto.log
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/zz/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/zz/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/zz/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/zz/bench.log | cut -c1-300; exit $rc
