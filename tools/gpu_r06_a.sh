#!/bin/bash
# GPU session (round 6): -m gpu tests, then the leaf_pairs A/B (tools/gpu_ab_pairs.sh)
set -u
mkdir -p gpurun_out/r06_c
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r06_c/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 12 gpurun_out/r06_c/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_OUT=r06_c bash tools/gpu_ab_pairs.sh
