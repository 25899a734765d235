#!/bin/bash
# VALU / MFMA busy and HBM traffic of the CWT workload (default pipelined schedule, cfg3 shape):
# the north_star asks for MFMA-busy evidence on the FFT path.  Separate passes, kernel trace
# only.  Usage: tools/pmc_cwt_busy.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-b}"
O="$R/gpurun_out/pmccwtbusy_$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_ANY" \
            "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/p$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload cwt --steps 1 --warmup 1 --no-cpu-baseline --no-check > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/p$i.log"; exit $rc; }
done
