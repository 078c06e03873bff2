#!/bin/bash
# GPU session (round 6, i): -m gpu tests; same-box A/B of the fma Hermite weights and the shared upper-lane
# shift of the perlin corner offsets (lib) against the tree before them (lib/ab/librtgpu_pre4.so) on config 3
set -u
OUT=gpurun_out/r06_i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L="lib=raytracing-practice_amd/lib/librtgpu.so,pre=raytracing-practice_amd/lib/ab/librtgpu_pre4.so"
timeout -k 10 300 python3 tools/ab_schedule.py --libs $L --rounds 6 --scene earth_perlin \
  --variants 'pre@0:0:0,lib@0:0:0' > $OUT/c3.json 2> $OUT/c3.err
rc=$?
echo "== c3 rc=$rc"; python3 tools/abshow.py $OUT/c3.json 2>/dev/null || tail -5 $OUT/c3.err
exit $rc
