#!/bin/bash
# GPU session (round 6, e): -m gpu tests; config 3's LDS bank conflicts attributed by layout — the shipped
# library against lib/ab/librtgpu_perlinglobal.so (the same tree with the textured LDS kernel's Perlin
# tables read through L1/L2 instead of LDS; built by hand from a patched copy of csrc/, not shipped):
# same-box A/B timing, then one SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS pass per library
set -u
OUT=gpurun_out/r06_e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 8 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L="lib=raytracing-practice_amd/lib/librtgpu.so,pg=raytracing-practice_amd/lib/ab/librtgpu_perlinglobal.so"
timeout -k 10 300 python3 tools/ab_schedule.py --libs $L --rounds 4 --scene earth_perlin \
  --variants 'lib@0:0:0,pg@0:0:0' > $OUT/c3.json 2> $OUT/c3.err
rc=$?
echo "== c3 rc=$rc"; python3 tools/abshow.py $OUT/c3.json 2>/dev/null || tail -5 $OUT/c3.err
[ $rc -eq 0 ] || exit $rc
export RTG_DUAL=0
for v in lib pg; do
  if [ $v = pg ]; then export RTGPU_LIB=raytracing-practice_amd/lib/ab/librtgpu_perlinglobal.so; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -f csv -d $OUT/pmc_sq2_$v -o run -- \
    python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_sq2_$v.log 2>&1
  rc=$?
  echo "== pmc_sq2_$v rc=$rc"; tail -n 2 $OUT/pmc_sq2_$v.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -f csv -d $OUT/pmc_sq_$v -o run -- \
    python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_sq_$v.log 2>&1
  rc=$?
  echo "== pmc_sq_$v rc=$rc"; tail -n 2 $OUT/pmc_sq_$v.log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
