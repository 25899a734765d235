#!/bin/bash
# Counter passes over the CWT band kernel (cwt_band512) at cfg3 geometry, batch 64: where its
# wave cycles go (wait / issue-stall / active), VALU / MFMA / LDS / memory instruction counts.
# Usage: TAG [JW_CWT_BAND_V values...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/pmcband2_$1"; mkdir -p "$O"; shift
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES"
P3="GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
for v in "${@:-3}"; do
  i=1
  for P in "$P1" "$P2" "$P3"; do
    JW_CWT_BAND_V=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex cwt_band512 \
      -d "$O/v${v}_p$i" -o run --output-format csv -- python3 "$R/bench.py" --workload cwt --steps 1 \
      --warmup 1 --no-cpu-baseline --no-check --batch 64 > "$O/v${v}_p$i.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "v$v p$i rc=$rc"; tail -5 "$O/v${v}_p$i.log"; exit $rc; }
    python3 - "$O/v${v}_p$i/run_counter_collection.csv" "v$v p$i" <<'PY'
import csv, collections, sys
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], {k: f"{v:.4g}" for k, v in sorted(agg.items())})
PY
    i=$((i+1))
  done
done
