#!/bin/bash
# GPU session (round 6, w): HEAD check (smoke, bench.py --config 2) after the host-only tile-order knob; and the
# 64x1 shard tile (RTG_TILE_LW=6) for config 2's 8-GPU shards against 16x4 (profiles/r06_t: 96.8 ms summed)
set -u
OUT=gpurun_out/r06_w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py --config 2 > $OUT/bench_config2.log 2>&1 || { tail $OUT/bench_config2.log; exit 1; }
grep '^{' $OUT/bench_config2.log > $OUT/bench_config2.json
python3 -c "import json; d=json.load(open('$OUT/bench_config2.json')); print(d['value'], d['ms_per_step'], d['tile_order'], d['parity']['identical_frac'])"
RTG_TILE_LW=6 timeout -k 10 300 python3 tools/shard_probe.py --config 2 --reps 2 --ns 1,8 --prepare > $OUT/c2_strided_lw6.json 2> $OUT/c2_strided_lw6.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/c2_strided_lw6.json')); print({k: (v['sum_kernel_ms'], v['max_wall_ms'], v['efficiency_vs_n1']) for k, v in d['per_n'].items()})"
