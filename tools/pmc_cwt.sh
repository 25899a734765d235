#!/bin/bash
# PMC passes over the CWT bench (separate passes, kernel trace only).  Usage: tools/pmc_cwt.sh TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
mkdir -p "$R/gpurun_out/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $ctrs -d "$R/gpurun_out/pmc_$TAG/p$i" -o run \
      --output-format csv -- python3 "$R/bench.py" --workload cwt --no-cpu-baseline --no-check "$@" \
      > "$R/gpurun_out/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_$TAG/p$i.log"; exit $rc; fi
done
