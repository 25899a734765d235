# round-4 call s: inverse levels at 512 x 2048 (product) -- STRICT parity, then AUTO timing
# against the square split everywhere (JW_AUTO_R=1024)
mkdir -p gpurun_out/s
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py tests/test_jni_glue_gpu.py tests/test_host_pipeline_gpu.py > gpurun_out/s/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/s/pytest.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/s
for rep in 1 2; do
  for R in 0 1024; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JW_AUTO_R=$R timeout -k 10 300 python3 tools/modwt_time.py --method auto --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > $O/one.log 2>&1 || { echo "R=$R failed"; tail -5 $O/one.log; exit 1; }
      echo "R=$R $wn $(tail -1 $O/one.log | cut -c1-220)" | tee -a $O/ab.log
    done
  done
done
