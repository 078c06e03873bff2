#!/bin/bash
# tools/gpu_profile_configs.sh OUTDIR [configs...] — rocprofv3 kernel trace + PMC passes (tools/profile.sh)
# of bench.py --config N for each config, into gpurun_out/OUTDIR/prof_cN (through gpurun, repo root).
set -u
OUT=gpurun_out/${1:-prof}
shift || true
for c in ${*:-2 3 4 5}; do
  echo "=== config $c"
  PROF_OUT=$OUT/prof_c$c STEPS=2 bash tools/profile.sh --config "$c" || exit $?
done
exit 0
