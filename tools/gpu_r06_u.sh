#!/bin/bash
# GPU session (round 6, u): the tile-cost probe's sample count (RTG_TILE_ORDER_SPP 4 default / 16 / 1) against
# the 8-GPU shard's tail (config 2: 90 % of a 1/8 shard's waves end within 0.18 ms, the last 10 % 0.36 ms later,
# profiles/r06_s); shard probe sums and maxima at N = 1, 8 for configs 2 and 3
set -u
OUT=gpurun_out/r06_u
mkdir -p $OUT
export TMPDIR=/tmp
sp() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 tools/shard_probe.py --reps 3 --ns 1,8 --prepare "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; python3 -c "import json; d=json.load(open('$OUT/$n.json')); print({k: (v['sum_kernel_ms'], v['max_wall_ms'], v['efficiency_vs_n1']) for k, v in d['per_n'].items()})" || tail -3 $OUT/$n.err
  return $rc
}
for c in 2 3; do
  for k in 4 16 1; do
    RTG_TILE_ORDER_SPP=$k sp c${c}_spp$k --config $c || exit $?
  done
done
