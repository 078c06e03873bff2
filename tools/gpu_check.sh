#!/bin/bash
# tools/gpu_check.sh — GPU-box validation run (invoked through gpurun from the repo root).
#   smoke -> pytest -m gpu -> bench; stops at the first step that does not end normally.
# Usage: tools/gpu_check.sh [bench args...]
set -u
mkdir -p gpurun_out
step() {  # name timeout-seconds command...
  local name=$1 t=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
step smoke 400 python3 -c "import __graft_entry__ as g; g.smoke()" || exit $?
step gpu_tests 1200 python3 -m pytest tests -m gpu -q -rf --timeout 600
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 900 python3 bench.py "$@" || exit $?
grep '^{' gpurun_out/bench.log > gpurun_out/bench.json
exit 0
