#!/bin/bash
# GPU session (round 6): leaf_pairs A/B on configs 2, 5 and 3 (same box, alternating rounds), counts and
# schedule diagnostics of both builds. The prototype left the product (measured rejection, profiles/r06_pairs):
# git apply tools/experiments/leaf_pairs.patch, then make -C raytracing-practice_amd && tools/build_ab.sh nopairs -DRTG_LEAF_PAIRS=0
set -u
OUT=gpurun_out/${AB_OUT:-r06_pairs}
mkdir -p $OUT
export TMPDIR=/tmp
L="lib=raytracing-practice_amd/lib/librtgpu.so,nopairs=raytracing-practice_amd/lib/ab/librtgpu_nopairs.so"
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  echo "== $n"
  timeout -k 10 $t python3 tools/ab_schedule.py --libs $L "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
dg() {  # name timeout lib args...
  local n=$1 t=$2 l=$3; shift 3
  timeout -k 10 $t python3 tools/diag.py --lib $l "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; grep -E "lane_util|kernel_ms|cycles_per|leaf_" $OUT/$n.json | tr -d '\n'; echo
  return $rc
}
ab c2 300 --rounds 4 --count --variants 'nopairs@0:0:0,lib@0:0:0' || exit $?
ab c5 600 --rounds 2 --count --grid 500 --width 3840 --spp 1000 --variants 'nopairs@0:0:0,lib@0:0:0' || exit $?
ab c3 300 --rounds 3 --scene earth_perlin --variants 'nopairs@0:0:0,lib@0:0:0' || exit $?
dg diag_c2_pairs 200 raytracing-practice_amd/lib/librtgpu.so --batches 0 || exit $?
dg diag_c2_nopairs 200 raytracing-practice_amd/lib/ab/librtgpu_nopairs.so --batches 0 || exit $?
dg diag_c5_pairs 300 raytracing-practice_amd/lib/librtgpu.so --grid 500 --width 3840 --spp 1000 --batches 0 || exit $?
dg diag_c5_nopairs 300 raytracing-practice_amd/lib/ab/librtgpu_nopairs.so --grid 500 --width 3840 --spp 1000 --batches 0 || exit $?
