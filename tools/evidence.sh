#!/bin/bash
# The one evidence script: every number in DESIGN.md §7 comes from a pass of this script
# (profiles/r05/INDEX.md maps each number to its file).  Each GPU step runs under its own time
# limit, steps are chained, and the script stops at the first failure.
#
# Usage: tools/evidence.sh TAG PASS [WORKLOAD] [extra bench.py args...]
#   PASS      tests   the -m gpu suite (TESTS="tests/test_x.py ..." narrows it)
#             smoke   __graft_entry__.smoke()
#             bench   one bench.py line per workload (bench_all: every BASELINE config)
#             stats   rocprofv3 --kernel-trace --stats of the workload's timed launches
#             traffic FETCH_SIZE and WRITE_SIZE passes (separate runs, kernel trace only)
#             sq      SQ activity / VALU / MFMA-busy / LDS counters (one pass, kernel trace only)
#             ab      same-box A/B of library builds (LIBS="base v1 ..", REPS rounds)
#             envab   same-box A/B of environment settings (ENVS="base;K=V;K=V K2=V2", REPS
#                     rounds; STATS=1 adds a kernel trace per setting)
#             final   tests, smoke, bench_all, then stats + traffic of modwt and cwt
#   WORKLOAD  modwt (headline, default) | sym8 (cfg5) | cwt (cfg3) | fwt2d (cfg4) |
#             auto (JWave's default path: AUTO STRICT db4 J=8, 128 x 2^20, tools/modwt_time.py) |
#             fft (JWave's FFT alone, 128 x 2^20, tools/fft_time.py; JW_JFFT_3PASS_MIN=1048576 for
#             the three-pass split)
# Output: gpurun_out/TAG/ (copy what is judged into profiles/rNN/).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:?tag}"; PASS="${2:?pass}"; W="${3:-modwt}"
shift $(( $# < 3 ? $# : 3 ))
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
export TMPDIR=/tmp

cmd_for() {  # the program one workload runs (after rocprofv3's --, or on its own)
  case "$1" in
    modwt) echo "python3 $R/bench.py --no-cpu-baseline --no-check --no-alt --steps 3 --warmup 1" ;;
    sym8)  echo "python3 $R/bench.py --wavelet Symlet8 --levels 6 --no-cpu-baseline --no-check --no-alt --steps 3 --warmup 1" ;;
    cwt)   echo "python3 $R/bench.py --workload cwt --no-cpu-baseline --no-check --steps 3 --warmup 1" ;;
    fwt2d) echo "python3 $R/bench.py --workload fwt2d --no-cpu-baseline --no-check --no-alt --steps 3 --warmup 1" ;;
    auto)  echo "python3 $R/tools/modwt_time.py --method auto --arith strict --batch 128 --reps 3" ;;
    fft)   echo "python3 $R/tools/fft_time.py --n 1048576 --batch 128 --reps 3" ;;
    *) echo "unknown workload $1" >&2; exit 2 ;;
  esac
}

step() {  # name, seconds, command...: run, log, stop the script on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -8 "$O/$name.log"; exit $rc; }
}

prof() {  # name, rocprof args..., --, workload
  local name=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done
  shift
  local c; c=$(cmd_for "$1") || exit 2; shift
  # shellcheck disable=SC2086
  (cd /tmp && timeout -s KILL 300 rocprofv3 "${args[@]}" -d "$O/$name" -o run --output-format csv \
      -- $c "$@" > "$O/$name.log" 2>&1)
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -8 "$O/$name.log"; exit $rc; }
}

SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_ANY"
SQ2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT"

run_pass() {
  local p=$1 w=$2; shift 2
  case "$p" in
    tests)
      # shellcheck disable=SC2086
      step "pytest" 1500 python -u -m pytest ${TESTS:-tests} -m gpu -q -x -p no:cacheprovider \
          --timeout 120 --timeout-method thread
      tail -2 "$O/pytest.log" ;;
    smoke)
      step "smoke" 300 python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 "$O/smoke.log" ;;
    bench)
      if [ "$w" = "all" ]; then
        : > "$O/bench_all.jsonl"
        for a in "--workload fwt2d --steps 5 --warmup 2" \
                 "--workload fwt2d --steps 5 --warmup 2 --arith strict --no-cpu-baseline" \
                 "--workload cwt --steps 3 --warmup 1" \
                 "--wavelet Symlet8 --levels 6 --no-cpu-baseline --no-alt" \
                 "--wavelet Symlet8 --levels 6 --global-batch 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-alt" \
                 ""; do
          # shellcheck disable=SC2086
          step "bench_one" 600 python bench.py $a
          grep '^{' "$O/bench_one.log" >> "$O/bench_all.jsonl"
        done
        cut -c1-200 "$O/bench_all.jsonl"
      elif [ "$w" = "auto" ]; then
        # shellcheck disable=SC2046
        step "bench_auto" 600 $(cmd_for auto) "$@"
        tail -2 "$O/bench_auto.log"
      else
        # shellcheck disable=SC2046
        step "bench_$w" 600 $(cmd_for "$w" | sed 's/--no-cpu-baseline --no-check//') "$@"
        grep '^{' "$O/bench_$w.log" | cut -c1-400
      fi ;;
    stats)   prof "stats_$w" --kernel-trace --stats -- "$w" "$@" ;;
    traffic)
      prof "fetch_$w" --kernel-trace --pmc FETCH_SIZE -- "$w" "$@"
      prof "write_$w" --kernel-trace --pmc WRITE_SIZE -- "$w" "$@" ;;
    sq)
      # shellcheck disable=SC2086
      prof "sq_$w" --kernel-trace --pmc $SQ -- "$w" "$@"
      # shellcheck disable=SC2086
      prof "sq2_$w" --kernel-trace --pmc $SQ2 -- "$w" "$@" ;;
    ab)
      # same-box A/B of library builds, alternating: LIBS="base v1 v2" (base = the product,
      # vN = jwave-pro_amd/ab/libjwave_hip_vN.so from tools/build_variant.sh), REPS rounds
      for rep in $(seq "${REPS:-2}"); do
        for L in ${LIBS:?LIBS}; do
          lib="$R/jwave-pro_amd/libjwave_hip.so"
          [ "$L" = base ] || lib="$R/jwave-pro_amd/ab/libjwave_hip_$L.so"
          # shellcheck disable=SC2046
          JWAVE_HIP_LIB="$lib" step "ab_${w}_${L}_$rep" 300 $(cmd_for "$w") "$@"
          grep '^{' "$O/ab_${w}_${L}_$rep.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d.get('roofline') or {}
keys = [k for k in list(d) + list(r) if k.endswith('_ms') or k in ('value', 'msamples_s')]
print('$L', {k: d.get(k, r.get(k)) for k in keys})" | tee -a "$O/ab_${w}.txt"
        done
      done ;;
    envab)
      # same-box A/B of environment settings, alternating: ENVS="base;JW_X=1;JW_X=1 JW_Y=0"
      # (base = no extra settings), REPS rounds; with STATS=1 also a kernel-trace per setting
      IFS=';' read -r -a sets <<< "${ENVS:?ENVS}"
      for rep in $(seq "${REPS:-2}"); do
        for i in "${!sets[@]}"; do
          e="${sets[$i]}"; [ "$e" = base ] && e=""
          # shellcheck disable=SC2046,SC2086
          timeout -k 10 300 env $e $(cmd_for "$w") "$@" > "$O/envab_${w}_${i}_$rep.log" 2>&1
          rc=$?; [ $rc -eq 0 ] || { echo "envab $i rc=$rc"; tail -8 "$O/envab_${w}_${i}_$rep.log"; exit $rc; }
          grep '^{' "$O/envab_${w}_${i}_$rep.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
r = d.get('roofline') or {}
keys = [k for k in list(d) + list(r) if k.endswith('_ms') or k in ('value', 'msamples_s')]
print('[${sets[$i]}]', {k: d.get(k, r.get(k)) for k in keys})" | tee -a "$O/envab_${w}.txt"
        done
      done
      if [ "${STATS:-0}" = 1 ]; then
        for i in "${!sets[@]}"; do
          e="${sets[$i]}"; [ "$e" = base ] && e=""
          # shellcheck disable=SC2086
          (if [ -n "$e" ]; then export $e; fi; prof "envstats_${w}_$i" --kernel-trace --stats -- "$w" "$@") || exit 1
        done
      fi ;;
    final)
      run_pass tests x
      run_pass smoke x
      run_pass bench all
      for x in modwt cwt; do run_pass stats $x; run_pass traffic $x; done ;;
    *) echo "unknown pass $p" >&2; exit 2 ;;
  esac
}

run_pass "$PASS" "$W" "$@"
echo "evidence $TAG $PASS $W done"
