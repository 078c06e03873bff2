#!/bin/bash
# tools/gpu_session.sh OUTDIR [configs...] — one GPU-box session (through gpurun, from the repo root):
#   pytest -m gpu, then bench.py --config N for each config (default: 2), each step under its own
#   time limit; stops at the first step that does not end normally. Results in gpurun_out/OUTDIR/.
set -u
OUT=gpurun_out/${1:-session}
shift || true
CONFIGS=${*:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout-seconds command...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "$OUT/$name.log"
  return $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
  rc=$?
  [ $rc -ne 0 ] && exit $rc
fi
for c in $CONFIGS; do
  step bench_config$c 900 python3 bench.py --config "$c" ${BENCH_ARGS:-} || exit $?
  grep '^{' "$OUT/bench_config$c.log" > "$OUT/bench_config$c.json"
done
exit 0
