#!/bin/bash
# GPU session (round 6, v): the final tree's benchmark frames of configs 2, 3 and 4 at full size and full spp,
# rendered in the prepared tile order (rtg_scene_prepare, as bench.py renders them), every pixel against
# cpu_ref32 on the box's 16 cores (tests/tools/full_frame_check.py), with the segment counts
set -u
OUT=gpurun_out/r06_v
mkdir -p $OUT
export TMPDIR=/tmp
ff() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u tests/tools/full_frame_check.py --prepare "$@" > $OUT/$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc"; grep -E '"(differing_pixels|identical_frac|segments_equal|gpu_tile_order|oracle_seconds)"' $OUT/$n.log
  return $rc
}
ff full_c2 300 || exit $?
ff full_c3 300 --scene earth_perlin --grid 0 || exit $?
ff full_c4 420 --scene cornell_box --grid 0 --width 800 --height 800 --spp 2000 --depth 100 || exit $?
