#!/bin/bash
# PMC passes (separate runs, kernel trace only) over one microbenchmark command:
#   pmc_run.sh TAG program [args...]   -> gpurun_out/pmc_TAG/p{1,2,3}/...
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
TAG="$1"; shift
mkdir -p "$R/gpurun_out/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
            "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE SQ_INSTS_SMEM" \
            "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$R/gpurun_out/pmc_$TAG/p$i" -o run \
      --output-format csv -- "$@" > "$R/gpurun_out/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_$TAG/p$i.log"; exit $rc; fi
done
