#!/bin/bash
# A/B timing of JWave's default path (AUTO STRICT, 128 x 2^20) under env knobs, alternating.
# Usage: tools/ab_auto.sh TAG "ENV=VAL ..." ["ENV=VAL ..." ...]   (first = baseline "")
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/ab_auto_$1"; shift; mkdir -p "$O"
CFGS=("" "$@")
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      env $cfg timeout -k 10 300 python3 "$R/tools/modwt_time.py" --method auto --arith strict \
        --batch 128 --reps 3 --wavelet $wn --levels $wl > "$O/one.log" 2>&1 || { tail -5 "$O/one.log"; exit 1; }
      echo "[$cfg] $(tail -1 "$O/one.log")" | tee -a "$O/ab.log"
    done
  done
done
