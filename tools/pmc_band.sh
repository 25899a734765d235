#!/bin/bash
# Counters of the CWT band kernel (cwt_band512) at the cfg3 shape, plus a kernel trace with
# only the narrowest bands (JW_CWT_BAND=8).  Separate passes, kernel trace only.
# Usage: tools/pmc_band.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-b}"
O="$R/gpurun_out/pmcband_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
B="--workload cwt --steps 1 --warmup 1 --no-cpu-baseline --no-check --batch 64"
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs --kernel-include-regex cwt_band512 \
    -d "$O/p$i" -o run --output-format csv -- python3 "$R/bench.py" $B > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/p$i.log"; exit $rc; }
done
for nb in 8 24 96; do
  JW_CWT_BAND=$nb timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/t$nb" -o run \
    --output-format csv -- python3 "$R/bench.py" $B > "$O/t$nb.log" 2>&1
  rc=$?; echo "trace $nb rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/t$nb.log"; exit $rc; }
done
