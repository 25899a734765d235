#!/bin/bash
# CWT band sums on the matrix cores (default) against the VALU (Gauss) form: cfg3 step time
# for both, then MFMA / VALU busy counters of cwt_band512 (batch 64).  Usage: TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/abmfma_$1"; mkdir -p "$O"
for m in 0 1; do
  JW_CWT_BAND_MFMA=$m timeout -k 10 120 python3 "$R/bench.py" --workload cwt --steps 5 --warmup 2 \
    --no-cpu-baseline --no-check > "$O/m$m.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "m $m rc=$rc"; tail -5 "$O/m$m.log"; exit $rc; }
  echo "mfma $m $(grep -h '^{' "$O/m$m.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  JW_CWT_BAND_MFMA=$m timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_SALU SQ_WAVES \
    --kernel-include-regex cwt_band512 -d "$O/p$m" -o run --output-format csv -- python3 "$R/bench.py" \
    --workload cwt --steps 1 --warmup 1 --no-cpu-baseline --no-check --batch 64 > "$O/p$m.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc $m rc=$rc"; tail -5 "$O/p$m.log"; exit $rc; }
  python3 - "$O/p$m/run_counter_collection.csv" "$m" <<'PY'
import csv, collections, sys
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
print("mfma", sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(agg.items())})
PY
done
