R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"
for spec in "JW_CWT_PIPE=0" "JW_CWT_PIPE=1" "JW_CWT_PIPE=1,JW_CWT_GROUP_MB=64" "JW_CWT_PIPE=1,JW_CWT_GROUP_MB=32" "JW_CWT_PIPE=1,JW_CWT_GROUP_MB=256"; do
  env $(echo "$spec" | tr ',' ' ') timeout -k 10 300 python bench.py --workload cwt --steps 3 --warmup 1 --no-cpu-baseline --no-check > /tmp/c.json 2>/dev/null || { echo "fail $spec"; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/c.json').read().strip().splitlines()[-1]); print('$spec', d['value'], d['ms_per_step'])"
done
