#!/bin/bash
# Summary of tools/pmc_band.sh output.  Usage: tools/pmc_band_summary.sh TAG
D=gpurun_out/pmcband_$1
for t in t8 t24 t96; do
  echo "== $t step_ms $(grep -h '^{' $D/$t.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
  python3 -c "
import csv
for r in csv.DictReader(open('$D/$t/run_kernel_stats.csv')):
    if 'band512' in r['Name'] or 'pass512_two' in r['Name']: print(r['Name'][:40], r['Calls'], r['AverageNs'], r['TotalDurationNs'])
"
done
python3 - "$D" <<'PY'
import csv, collections, sys
for p in ['p1', 'p2', 'p3', 'p4']:
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f'{sys.argv[1]}/{p}/run_counter_collection.csv')):
        agg[r['Counter_Name']] += float(r['Counter_Value'])
    print(p, dict(agg))
PY
