#!/bin/bash
# A/B two builds of the engine on one box: tools/ab_so.sh TAG "bench args" (needs
# jwave-pro_amd/libjwave_hip_old.so and libjwave_hip_new.so); runs old, new, old, new.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG="$1"; ARGS="$2"
for v in old new old new; do
  cp jwave-pro_amd/libjwave_hip_$v.so jwave-pro_amd/libjwave_hip.so
  timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > gpurun_out/abso_${TAG}_$v.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -3 gpurun_out/abso_${TAG}_$v.log; exit $rc; fi
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abso_${TAG}_$v.log') if l.startswith('{')][-1])
r=d['roofline']; print('$v', d['value'], d['ms_per_step'], {k: r[k] for k in r if k.endswith('_ms')})"
done
