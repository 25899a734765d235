#!/bin/bash
# A/B of the product library against experimental builds on cfg3 (CWT Morlet, 64 scales, N=2^18 x 256),
# alternating.  Usage: tools/ab_cwt_libs.sh TAG NAME [NAME ...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O="gpurun_out/ab_cwt_libs_$1"; shift; mkdir -p "$O"
LIBS=("libjwave_hip.so")
for n in "$@"; do LIBS+=("ab/libjwave_hip_$n.so"); done
for rep in 1 2; do
  for lib in "${LIBS[@]}"; do
    for ar in fma; do
      JWAVE_HIP_LIB=$R/jwave-pro_amd/$lib timeout -k 10 300 python3 bench.py --workload cwt \
        --steps 3 --warmup 1 --no-cpu-baseline --no-check > "$O/one.log" 2>&1 \
        || { echo "$lib failed"; tail -5 "$O/one.log"; exit 1; }
      python3 -c "
import json
d=json.loads([l for l in open('$O/one.log') if l.startswith('{')][-1])
print('$lib', '$ar', d['value'], d['ms_per_step'], {k: v for k, v in d['roofline'].items() if k.endswith('_ms')})" | tee -a "$O/ab.log"
    done
  done
done
