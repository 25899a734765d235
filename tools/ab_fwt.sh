#!/bin/bash
# FWT parity tests, then the fwt2d bench A/B over an env knob: tools/ab_fwt.sh TAG VAR "v1 v2 ..."
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="$1"; VAR="$2"; VALS="$3"; shift 3
timeout -k 10 400 python -u -m pytest tests/test_fwt_gpu.py tests/test_wpt_gpu.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/abf_${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/abf_${TAG}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abf_${TAG}_$v -o run --output-format csv -- python3 bench.py --workload fwt2d --no-cpu-baseline "$@" > gpurun_out/abf_${TAG}_$v.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "bench $v rc=$rc"; tail -5 gpurun_out/abf_${TAG}_$v.log; exit $rc; fi
  python3 - "$v" "gpurun_out/abf_${TAG}_$v" <<'PY'
import csv, glob, json, sys
v, d = sys.argv[1], sys.argv[2]
line = [l for l in open(d + ".log") if l.startswith("{")][-1]
j = json.loads(line)
print(v, "step", j["ms_per_step"], "value", j["value"], j.get("spot_check_vs_oracle"))
for r in csv.DictReader(open(glob.glob(d + "/*kernel_stats.csv")[0])):
    if "fwt" in r["Name"]:
        print("   %-60s %4s %8.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
done
