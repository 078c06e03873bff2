#!/bin/bash
# GPU session (round 6, o): the per-rank work of N = 1, 2, 4, 8 GPU frames on one GPU (tools/shard_probe.py:
# the interleaved row shards bench.py deals, rendered one after another) for configs 2-5 with the final
# kernels: the kernel-side strong-scaling efficiency N * max(shard) / frame the driver's 8-GPU run will see
set -u
OUT=gpurun_out/r06_o
mkdir -p $OUT
export TMPDIR=/tmp
for c in 2 3 4 5; do
  timeout -k 10 300 python3 tools/shard_probe.py --config $c --reps 2 > $OUT/shard_c$c.json 2> $OUT/shard_c$c.err
  rc=$?
  echo "== config $c rc=$rc"; tail -c 600 $OUT/shard_c$c.json
  if [ $rc -ne 0 ]; then tail -5 $OUT/shard_c$c.err; exit $rc; fi
done
