#!/bin/bash
# GPU session (round 6, s): per-wave timelines of rank 0's shard with the tile order (tools/wave_trace.py
# --prepare) for configs 2 and 3 at N = 1 and 8: what is left of the 8-GPU shard's time beyond 1/8 of the frame
set -u
OUT=gpurun_out/r06_s
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name args...
  local n=$1; shift
  timeout -k 10 200 python3 tools/wave_trace.py "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  echo "== $n rc=$rc"; cat $OUT/$n.json
  return $rc
}
for p in "" "--prepare"; do
  run c2_n1${p:+_prep} --spp 500 $p || exit $?
  run c2_n8${p:+_prep} --spp 500 --shard-of 8 $p || exit $?
  run c3_n8${p:+_prep} --scene earth_perlin --grid 0 --spp 500 --shard-of 8 $p || exit $?
done
