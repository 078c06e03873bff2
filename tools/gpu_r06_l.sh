#!/bin/bash
# GPU session (round 6, l): -m gpu tests; same-box A/B of the child codes carried in the 4-wide sort keys
# (LdsStack16 trees: the code row read with the box rows, no LDS read after the sort) (lib) against the
# tree before it (lib/ab/librtgpu_pre7.so) on configs 2 and 4, frames compared; the counter it should move
# is the wave-time share waiting (SQ_WAIT_ANY 0.31 on config 2)
set -u
OUT=gpurun_out/r06_l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L="lib=raytracing-practice_amd/lib/librtgpu.so,pre=raytracing-practice_amd/lib/ab/librtgpu_pre7.so"
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 tools/ab_schedule.py --libs $L "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
ab c2 300 --rounds 4 --count --variants 'pre@0:0:0,lib@0:0:0' || exit $?
ab c4 300 --rounds 3 --count --scene cornell_box --width 800 --height 800 --spp 2000 --depth 100 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
