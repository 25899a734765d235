#!/bin/bash
# FWT row reverse with two pairs per lane (new, the product) against one pair per lane (old,
# jwave-pro_amd/ab/libjwave_hip_old.so built with -DJW_REV_PAIRS2=0): FWT/WPT parity of the
# product, then cfg4 step times in both contracts, alternating, and the row reverse's average
# duration under rocprofv3.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
O=gpurun_out/ab_revpairs; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fwt_gpu.py tests/test_wpt_gpu.py -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for arith in fma strict; do
  for v in old new old new; do
    JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_$v.so timeout -k 10 200 python3 bench.py \
      --workload fwt2d --steps 5 --warmup 2 --arith $arith --no-cpu-baseline --no-check > $O/t.log 2>&1 \
      || { echo "bench rc=$?"; tail -3 $O/t.log; exit 1; }
    echo "$arith $v $(grep '^{' $O/t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  for arith in fma strict; do
    JWAVE_HIP_LIB=$R/jwave-pro_amd/ab/libjwave_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d "$R/$O/p_${v}_$arith" -o run --output-format csv -- python3 "$R/bench.py" --workload fwt2d \
      --steps 2 --warmup 1 --arith $arith --no-cpu-baseline --no-check > "$R/$O/p_${v}_$arith.log" 2>&1 \
      || { echo "prof rc=$?"; exit 1; }
    python3 - "$R/$O/p_${v}_$arith/run_kernel_stats.csv" "$v $arith" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fwt_" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0][-48:], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
  done
done
