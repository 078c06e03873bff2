#!/bin/bash
# tools/profile.sh — rocprofv3 evidence for the render kernel (run through gpurun from the repo root).
#   1. kernel trace + stats of the default bench workload (durations to compare with bench.py)
#   2. separate PMC passes (never combined with other tracing): HBM bytes, then SQ/TCP/TCC counters
# Outputs land in gpurun_out/prof/; copy the summaries worth keeping into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p "$OUT"
BENCH=(python3 bench.py --steps "${STEPS:-3}" --warmup 1 --no-cpu-baseline "$@")
PMC_BENCH=(python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@")
# counter collection serialises dispatches: a dual launch's second persistent kernel
# would only start after the first had taken all the work, so the PMC passes profile the single
# 16-wave launch (RTG_DUAL=0); the trace pass above times the shipped dual launch
run() {  # name timeout rocprofv3-args...
  local name=$1 t=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  return $rc
}
run trace 600 --kernel-trace --stats -S --summary-output-file summary \
    -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" || exit $?
export RTG_DUAL=0
run pmc_fetch 600 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- "${PMC_BENCH[@]}" || exit $?
run pmc_write 600 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- "${PMC_BENCH[@]}" || exit $?
run pmc_sq 600 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU \
    -f csv -d "$OUT/pmc_sq" -o run -- "${PMC_BENCH[@]}" || exit $?
run pmc_sq2 600 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/pmc_sq2" -o run -- "${PMC_BENCH[@]}" || exit $?
run pmc_cache 600 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum \
    -f csv -d "$OUT/pmc_cache" -o run -- "${PMC_BENCH[@]}" || exit $?
run pmc_ta 600 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/pmc_ta" -o run -- "${PMC_BENCH[@]}" || exit $?
exit 0
