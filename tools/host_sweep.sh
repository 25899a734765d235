#!/bin/bash
# JW_HOST staging A/B: copy threads x bounce-buffer size (tools/host_time.py)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
OUT=gpurun_out/host_sweep_${1:-a}.log
: > $OUT
for T in 6 8 10 12; do
  for P in 32 64 128; do
    JW_COPY_THREADS=$T JW_PIN_MB=$P timeout -k 10 120 python tools/host_time.py --reps 4 >> $OUT 2>&1 || exit $?
  done
done
python3 -c "import json,sys; [print(d[\"copy_threads\"], d[\"pin_mb\"], d[\"ms_per_fwd_inv\"], d[\"msamples_s\"], d[\"bit_identical_to_device_path\"]) for d in (json.loads(l) for l in open(sys.argv[1]) if l.startswith(\"{\"))]" $OUT
