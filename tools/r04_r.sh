# round-4 call r: AUTO STRICT column split (JW_AUTO_R = forward pass-1 column length) at N = 2^20:
# parity at each split, then timing, alternating
mkdir -p gpurun_out/r
for R in 512 2048; do
  JW_AUTO_R=$R timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_modwt_strict_gpu.py -k "full_size or bit_exact_vs_reference or fft_method_bit_exact" > gpurun_out/r/pytest_R$R.log 2>&1; rc=$?; echo "R=$R pytest rc=$rc"; tail -1 gpurun_out/r/pytest_R$R.log; [ $rc -eq 0 ] || exit $rc
done
O=gpurun_out/r
for rep in 1 2; do
  for R in 1024 512 2048; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JW_AUTO_R=$R timeout -k 10 300 python3 tools/modwt_time.py --method auto --arith strict --batch 128 --reps 3 --wavelet $wn --levels $wl > $O/one.log 2>&1 || { echo "R=$R failed"; tail -5 $O/one.log; exit 1; }
      echo "R=$R $wn $(tail -1 $O/one.log | cut -c1-220)" | tee -a $O/ab.log
    done
  done
done
