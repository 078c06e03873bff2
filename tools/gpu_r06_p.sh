#!/bin/bash
# GPU session (round 6, p): per-wave timelines (tools/wave_trace.py: start / end spread, waves alive per
# tenth of the kernel) of rank 0's shard at N = 1 and 8 for configs 3 and 2: where the 8-GPU shard's time
# beyond 1/8 of the frame goes (tools/shard_probe.py: config 3 N = 8 efficiency 0.73, config 2 0.91)
set -u
OUT=gpurun_out/r06_p
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python3 tools/wave_trace.py "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; cat $OUT/$n.json
  return $rc
}
run c3_n1 --scene earth_perlin --grid 0 --spp 500 || exit $?
run c3_n8 --scene earth_perlin --grid 0 --spp 500 --shard-of 8 || exit $?
run c2_n1 --spp 500 || exit $?
run c2_n8 --spp 500 --shard-of 8 || exit $?
