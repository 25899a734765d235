#!/bin/bash
# PMC passes (separate passes, kernel trace only) over any bench invocation.
# Usage: tools/pmc_any.sh TAG [bench args...]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; shift
mkdir -p "$R/gpurun_out/pmc_$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
            "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  case " ${PMC_PASSES:-1 2 3 4} " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $ctrs -d "$R/gpurun_out/pmc_$TAG/p$i" -o run \
      --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-check "$@" \
      > "$R/gpurun_out/pmc_$TAG/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$R/gpurun_out/pmc_$TAG/p$i.log"; exit $rc; fi
done
