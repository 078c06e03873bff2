#!/bin/bash
# GPU session (round 6, t): why an 8-GPU shard's waves run ~10 % longer per unit of work than the full frame's
# (profiles/r06_s: config 2's 1/8 shard, median wave end 12.57 ms against 91.4 / 8 = 11.4): ray coherence of the
# strided shard's tiles? Sum of the 8 shards' kernel times against the frame's, with the tile order, for the
# interleaved layout (16x4 tiles: 16 columns x 4 shard rows 8 image rows apart), interleaved with 8x8 and 32x2
# tiles (RTG_TILE_LW 3 / 5), and contiguous row blocks (8x8 tiles of image pixels; unbalanced, sum only)
set -u
OUT=gpurun_out/r06_t
mkdir -p $OUT
export TMPDIR=/tmp
sp() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 tools/shard_probe.py --reps 2 --ns 1,8 --prepare "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 -c "import json; d=json.load(open('$OUT/$n.json')); print({k: (v['sum_kernel_ms'], v['max_wall_ms'], v['efficiency_vs_n1']) for k, v in d['per_n'].items()})" || tail -3 $OUT/$n.err
  return $rc
}
for c in 2 3; do
  sp c${c}_strided --config $c || exit $?
  RTG_TILE_LW=3 sp c${c}_strided_lw3 --config $c || exit $?
  RTG_TILE_LW=5 sp c${c}_strided_lw5 --config $c || exit $?
  sp c${c}_contig --config $c --layout contig || exit $?
done
