#!/bin/bash
# GPU session (round 6, n): -m gpu tests; same-box A/B of the shared scatter steps (metal's and the
# dielectric's unit vector, and the first draw of every drawing lane, run once per shading phase instead of
# once per material branch; bit-identical by construction) (lib) against the tree before it
# (lib/ab/librtgpu_pre7.so) on configs 2 and 5 (both hold all three materials); frames compared.
# Prediction: -2 .. -3 % of the VALU instructions of config 2 (~38 per shading phase)
set -u
OUT=gpurun_out/r06_n
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
ab c2 300 --rounds 6 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
ab c5 400 --rounds 3 --grid 500 --width 3840 --spp 250 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
