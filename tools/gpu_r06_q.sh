#!/bin/bash
# GPU session (round 6, q): -m gpu tests (incl. test_tile_order_keeps_the_frame); same-box A/B of the
# cost-ordered tile hand-out (rtg_scene_prepare's tile-cost probe): the tree before it (pre7), this library
# with RTG_TILE_ORDER=0 (tile-major) and with the order, all prepared, configs 2-5 at N = 1; then the N = 8
# shards (tools/shard_probe.py) with and without the per-shard prepare. Prediction: the 8-GPU shards' tails
# shrink (config 3 efficiency 0.73 -> ~0.9, config 2 0.91 -> ~0.95), N = 1 within +-1 %
set -u
OUT=gpurun_out/r06_q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L="lib=raytracing-practice_amd/lib/librtgpu.so,pre=raytracing-practice_amd/lib/ab/librtgpu_pre7.so"
V='pre@0:0:0,lib@0:0:0!RTG_TILE_ORDER=0,lib@0:0:0'
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 tools/ab_schedule.py --libs $L --prepare "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
ab c2 300 --rounds 4 --variants "$V" || exit $?
ab c3 300 --rounds 4 --scene earth_perlin --variants "$V" || exit $?
ab c4 300 --rounds 3 --scene cornell_box --width 800 --height 800 --spp 2000 --depth 100 --variants "$V" || exit $?
ab c5 400 --rounds 3 --grid 500 --width 3840 --spp 250 --variants "$V" || exit $?
for c in 2 3 4 5; do
  for p in "" "--prepare"; do
    n=shard_c$c${p:+_prep}
    timeout -k 10 300 python3 tools/shard_probe.py --config $c --reps 2 --ns 1,8 $p > $OUT/$n.json 2> $OUT/$n.err
    rc=$?
    echo "== $n rc=$rc"; python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); print({k: (v['max_wall_ms'], v['efficiency_vs_n1']) for k, v in d['per_n'].items()})" || tail -3 $OUT/$n.err
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
