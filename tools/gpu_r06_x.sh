#!/bin/bash
# GPU session (round 6, x): config 5's launch tail (wave timelines at N = 1 and 8), and the tile order by 8x8-tile
# blocks (RTG_TILE_ORDER=2: blocks ranked by cost, tiles in raster order inside, also on the treelet schedule)
# against tile-major on config 5 and against the per-tile order on config 2; config 5's 8-GPU shards with it
set -u
OUT=gpurun_out/r06_x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/wave_trace.py --grid 500 --width 3840 --spp 1000 > $OUT/c5_n1.json 2> $OUT/c5_n1.err || exit 1
cat $OUT/c5_n1.json
timeout -k 10 300 python3 tools/wave_trace.py --grid 500 --width 3840 --spp 1000 --shard-of 8 > $OUT/c5_n8.json 2> $OUT/c5_n8.err || exit 1
cat $OUT/c5_n8.json
ab() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 tools/ab_schedule.py --prepare "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 tools/abshow.py $OUT/$n.json 2>/dev/null || tail -5 $OUT/$n.err
  return $rc
}
ab c5 500 --rounds 3 --grid 500 --width 3840 --spp 500 --variants 'lib@0:0:0!RTG_TILE_ORDER=0,lib@0:0:0!RTG_TILE_ORDER=2' || exit $?
ab c2 300 --rounds 4 --variants 'lib@0:0:0,lib@0:0:0!RTG_TILE_ORDER=2' || exit $?
RTG_TILE_ORDER=2 timeout -k 10 400 python3 tools/shard_probe.py --config 5 --reps 2 --ns 1,8 --prepare > $OUT/shard_c5_blocks.json 2> $OUT/shard_c5_blocks.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/shard_c5_blocks.json')); print({k: (v['sum_kernel_ms'], v['max_wall_ms'], v['efficiency_vs_n1']) for k, v in d['per_n'].items()})"
