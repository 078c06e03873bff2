#!/bin/bash
# tools/gpu_r05.sh OUTDIR STEP... — one GPU-box session (through gpurun, from the repo root). Steps:
#   tests           pytest -m gpu (failures reported, the session goes on; a crash or timeout ends it)
#   bench:N         bench.py --config N (BENCH_ARGS appended)
#   run:NAME:CMD    any command ('+' for spaces), NAME.log
#   testlib:LIB:EXPR  the GPU tests matching -k EXPR against another build (RTGPU_LIB=LIB); failures
#                   are the expected outcome of a negative control, so they do not end the session
#   ab:NAME:ARGS    tools/ab_schedule.py with ARGS (spaces as '+')
# Each step runs under its own time limit; results in gpurun_out/OUTDIR/.
set -u
OUT=gpurun_out/${1:-session}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout-seconds command...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 8 "$OUT/$name.log"
  return $rc
}
for s in "$@"; do
  case $s in
    tests)
      step gpu_tests 900 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
      rc=$?
      [ $rc -gt 1 ] && exit $rc ;;
    testk:*)  # testk:EXPR — the GPU tests matching -k EXPR ('+' for spaces)
      expr=${s#testk:}
      step gpu_tests_k 600 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k "${expr//+/ }"
      rc=$?
      [ $rc -gt 1 ] && exit $rc ;;
    bench:*)
      c=${s#bench:}
      step bench_config$c 700 python3 bench.py --config "$c" ${BENCH_ARGS:-} || exit $?
      grep '^{' "$OUT/bench_config$c.log" > "$OUT/bench_config$c.json" ;;
    testlib:*)
      rest=${s#testlib:}
      lib=${rest%%:*}
      expr=${rest#*:}
      RTGPU_LIB=$lib step gpu_tests_lib 600 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 \
        --timeout-method thread -k "${expr//+/ }"
      rc=$?
      [ $rc -gt 1 ] && exit $rc ;;
    prof:*)  # prof:NAME:CONFIG[:VAR=VAL^VAR=VAL] — tools/profile.sh (trace + PMC passes) of bench --config
      rest=${s#prof:}
      name=${rest%%:*}
      rest=${rest#*:}
      cfg=${rest%%:*}
      envs=""
      [ "$rest" != "$cfg" ] && envs=${rest#*:}
      echo "== prof_$name: config $cfg ${envs//^/ }"
      ( for kv in ${envs//^/ }; do export "$kv"; done
        PROF_OUT=$OUT/prof_$name STEPS=2 timeout -k 10 1000 bash tools/profile.sh --config "$cfg" ) > "$OUT/prof_$name.log" 2>&1
      rc=$?
      echo "== prof_$name rc=$rc"
      tail -n 4 "$OUT/prof_$name.log"
      [ $rc -ne 0 ] && exit $rc ;;
    benchenv:*)  # benchenv:NAME:CONFIG:VAR=VAL^... — bench.py --config CONFIG under extra environment
      rest=${s#benchenv:}
      name=${rest%%:*}
      rest=${rest#*:}
      cfg=${rest%%:*}
      envs=${rest#*:}
      ( for kv in ${envs//^/ }; do export "$kv"; done
        step "bench_$name" 700 python3 bench.py --config "$cfg" ${BENCH_ARGS:-} ) || exit $?
      grep '^{' "$OUT/bench_$name.log" > "$OUT/bench_$name.json" ;;
    benchargs:*)  # benchargs:NAME:ARGS — bench.py ARGS (spaces as '+')
      rest=${s#benchargs:}
      name=${rest%%:*}
      args=${rest#*:}
      step "bench_$name" 700 python3 bench.py ${args//+/ } || exit $?
      grep '^{' "$OUT/bench_$name.log" > "$OUT/bench_$name.json" ;;
    run:*)  # run:NAME:COMMAND — any command ('+' for spaces), output in NAME.log
      rest=${s#run:}
      name=${rest%%:*}
      cmd=${rest#*:}
      step "$name" 700 ${cmd//+/ } || exit $? ;;
    ab:*)
      rest=${s#ab:}
      name=${rest%%:*}
      args=${rest#*:}
      step "ab_$name" 700 python3 tools/ab_schedule.py ${args//+/ } || exit $? ;;
  esac
done
exit 0
