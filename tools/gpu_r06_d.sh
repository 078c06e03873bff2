#!/bin/bash
# GPU session (round 6): -m gpu tests; A/B of the round-6 kernel changes (no max_depth<=0 branch in the loop,
# 1 - v in the image branch, lane id at the end, sample and unit end in one register) against the tree
# before them (lib/ab/librtgpu_pre.so, commit cb3b6f4); config 5's rows 1050-2160 at full spp vs the oracle
set -u
OUT=gpurun_out/r06_d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L="lib=raytracing-practice_amd/lib/librtgpu.so,pre=raytracing-practice_amd/lib/ab/librtgpu_pre.so"
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 tools/ab_schedule.py --libs $L "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
ab c2 300 --rounds 4 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
ab c3 300 --rounds 4 --scene earth_perlin --variants 'pre@0:0:0,lib@0:0:0' || exit $?
ab c4 300 --rounds 3 --scene cornell_box --width 800 --height 800 --spp 2000 --depth 100 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
ab c5 400 --rounds 2 --grid 500 --width 3840 --spp 1000 --variants 'pre@0:0:0,lib@0:0:0' || exit $?
timeout -k 10 700 python3 -u tests/tools/full_frame_check.py --grid 500 --width 3840 --height 2160 --spp 1000 --block 46 --rows-from 1050 --rows-to 2160 > $OUT/full_c5b.log 2>&1
echo "full_c5b rc=$?"; tail -n 30 $OUT/full_c5b.log | grep -E '"rows"|differing_pixels|identical_frac|pixels_differing' 
