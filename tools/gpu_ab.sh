#!/bin/bash
# tools/gpu_ab.sh — GPU tests then an in-process schedule A/B (through gpurun from the repo root).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf --timeout 600 > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "gpu_tests rc=$rc"; tail -n 15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python3 tools/ab_schedule.py "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?
echo "ab rc=$rc"; cat gpurun_out/ab.json; tail -n 5 gpurun_out/ab.err
exit $rc
