#!/bin/bash
# SQ counter passes (separate runs, kernel trace only) over one program: wave-cycle breakdown
# (waits, issue, VALU / LDS activity) and the LDS pipe (busy, bank conflicts).
# Usage: tools/pmc_sq.sh TAG program [args...]   (program: bench.py or tools/modwt_time.py)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
O="$R/gpurun_out/pmcsq_$TAG"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
            "SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/p$i" -o run --output-format csv -- \
    python3 "$R/$@" > "$O/p$i.log" 2>&1
  rc=$?; echo "$TAG pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/p$i.log"; exit $rc; }
done
