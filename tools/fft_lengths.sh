#!/bin/bash
# MODWT FFT-path timings over lengths (tools/modwt_time.py), both arithmetic contracts, against
# DIRECT.  Usage: tools/fft_lengths.sh > gpurun_out/fft_lengths_TAG.log
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in 1048576 1000000 1048577 4194304 4000000; do
  for m in "direct fma" "fft fma" "fft strict" "auto strict"; do
    set -- $m
    timeout -k 10 120 python3 "$R/tools/modwt_time.py" --n $n --batch 4 --method $1 --arith $2 --reps 2 || exit 1
  done
done
