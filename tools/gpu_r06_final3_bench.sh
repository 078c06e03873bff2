#!/bin/bash
# Final round-6 records (tile order), part 2: smoke, pytest -m gpu, bench.py --config 2..5 on the final tree
# (the binding records of part 1 already regenerated) into gpurun_out/r06_final3
set -u
OUT=gpurun_out/r06_final3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
bash tools/gpu_session.sh r06_final3 2 3 4 5
