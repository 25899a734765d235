#!/bin/bash
# Experimental library build for on-box A/B (not the product): recompiles the listed sources with
# extra flags and links them with the product's other objects into jwave-pro_amd/ab/libjwave_hip_NAME.so.
# Usage: tools/build_variant.sh NAME "EXTRA FLAGS" src1.hip [src2.hip ...]   (run after make)
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R/jwave-pro_amd"
NAME=$1; FLAGS=$2; shift 2
mkdir -p ab/$NAME
objs=""
for o in build/*.o; do
  b=$(basename "$o" .o)          # e.g. jw_jfft.hip
  skip=0
  for src in "$@"; do [ "$b" = "$(basename "$src")" ] && skip=1; done
  [ $skip -eq 0 ] && objs="$objs $o"
done
for src in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -Wall \
    -I../include -Icsrc $FLAGS -x hip -c "csrc/$(basename "$src")" -o "ab/$NAME/$(basename "$src").o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "ab/libjwave_hip_$NAME.so" $objs ab/$NAME/*.o -l:libquadmath.so.0
echo "built ab/libjwave_hip_$NAME.so"
