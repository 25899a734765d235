#!/bin/bash
# A/B of environment knobs on one bench workload: step time per setting, then the kernels'
# average durations under rocprofv3 (kernel trace only).
# Usage: ab_env.sh TAG "BENCH ARGS" "ENV1=a ENV2=b" "ENV1=c" ...   (one quoted set per variant)
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/abenv_$1"; mkdir -p "$O"; shift
BA="$1"; shift
i=0
for v in "$@"; do
  env $v timeout -k 10 150 python3 "$R/bench.py" $BA --no-cpu-baseline --no-check > "$O/v$i.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[$v] rc=$rc"; tail -5 "$O/v$i.log"; exit $rc; }
  echo "[$v] $(grep -h '^{' "$O/v$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
  i=$((i+1))
done
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  export $v
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$O/p$i" -o run --output-format csv \
    -- python3 "$R/bench.py" $BA --steps 2 --warmup 1 --no-cpu-baseline --no-check > "$O/p$i.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "prof [$v] rc=$rc"; tail -5 "$O/p$i.log"; exit $rc; }
  for kv in $v; do unset "${kv%%=*}"; done
  python3 - "$O/p$i/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "synth" in r["Name"] or "copyBuffer" in r["Name"] or float(r["Percentage"]) < 1:
        continue
    print("[%s]" % sys.argv[2], r["Name"][:60], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
  i=$((i+1))
done
