#!/bin/bash
# lanes vs shade / leaf batch: one PMC pass over an in-process sweep (single 16-wave launch, RTG_DUAL=0)
set -u
OUT=gpurun_out/r03_h10
mkdir -p $OUT
export TMPDIR=/tmp
V='lib@0:1:0!RTG_DUAL=0,lib@0:16:0!RTG_DUAL=0,lib@0:32:0!RTG_DUAL=0,lib@0:48:0!RTG_DUAL=0,lib@0:56:0!RTG_DUAL=0,lib@0:64:0!RTG_DUAL=0,lib@0:48:1!RTG_DUAL=0,lib@0:48:32!RTG_DUAL=0'
timeout -k 10 300 python3 tools/ab_schedule.py --rounds 2 --variants "$V" > $OUT/ab_batches.json 2> $OUT/ab.err || { tail $OUT/ab.err; exit 1; }
python3 tools/abshow.py $OUT/ab_batches.json
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/pmc -o run -- python3 tools/ab_schedule.py --rounds 1 --variants "$V" > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
echo pmc done
