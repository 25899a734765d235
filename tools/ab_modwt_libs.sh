#!/bin/bash
# A/B of the product library against experimental builds on the MODWT benches: cfg2 (db4 J=8,
# the headline) and cfg5 (sym8 J=6), FMA, 1024 x 2^20, alternating; prints value and the
# forward / inverse kernel times.  Usage: tools/ab_modwt_libs.sh TAG NAME [NAME ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O="gpurun_out/ab_modwt_libs_$1"; shift; mkdir -p "$O"
LIBS=("libjwave_hip.so")
for n in "$@"; do LIBS+=("ab/libjwave_hip_$n.so"); done
for rep in ${REPS:-1 2}; do
  for lib in "${LIBS[@]}"; do
    for w in "Daubechies4 8" "Symlet8 6"; do
      read -r wn wl <<< "$w"
      JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 300 python3 bench.py --wavelet $wn \
        --levels $wl --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-check > "$O/one.log" 2>&1 \
        || { echo "$lib failed"; tail -5 "$O/one.log"; exit 1; }
      python3 -c "
import json
d=json.loads([l for l in open('$O/one.log') if l.startswith('{')][-1])
r=d['roofline']
print('$lib', '$wn', '$wl', d['value'], d['ms_per_step'], 'fwd', r.get('fwd_ms'), 'inv', r.get('inv_ms'), 'strict', d.get('other_arith', {}).get('value'), d.get('other_arith', {}).get('inv_ms'))" | tee -a "$O/ab.log"
    done
  done
done
