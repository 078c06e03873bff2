#!/bin/bash
# GPU session (round 6, m): timing-only probe of the draw cost — a 32-bit xorshift state (one VGPR, shifts
# and xors, no 64-bit multiplies) against the 64-bit LCG (lib/ab/librtgpu_pre7.so = the tree). Frames differ
# by construction (another random stream); compared by Mrays/s. Predicts the ceiling of a cheaper-RNG spec.
set -u
OUT=gpurun_out/r06_m
mkdir -p $OUT
export TMPDIR=/tmp
L="pre=raytracing-practice_amd/lib/ab/librtgpu_pre7.so,xs=raytracing-practice_amd/lib/ab/librtgpu_xs32.so"
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 tools/ab_schedule.py --libs $L "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
ab c2 300 --rounds 4 --variants 'pre@0:0:0,xs@0:0:0' || exit $?
ab c4 300 --rounds 3 --scene cornell_box --width 800 --height 800 --spp 2000 --depth 100 --variants 'pre@0:0:0,xs@0:0:0' || exit $?
ab c3 300 --rounds 3 --scene earth_perlin --variants 'pre@0:0:0,xs@0:0:0' || exit $?
ab c5 400 --rounds 3 --grid 500 --width 3840 --spp 250 --variants 'pre@0:0:0,xs@0:0:0' || exit $?
