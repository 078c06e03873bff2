#!/bin/bash
# Final round-6 records (tile order), part 1: rocprofv3 kernel trace + PMC passes (tools/profile.sh) of bench.py --config N
# for configs 2-5 on the final tree, into gpurun_out/r06_final3/prof_cN
set -u
mkdir -p gpurun_out/r06_final3
bash tools/gpu_profile_configs.sh r06_final3 2 3 4 5
