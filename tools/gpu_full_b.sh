set -o pipefail
mkdir -p gpurun_out/r06_b
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/r06_b/gpu_tests.log 2>&1 &&
timeout -k 10 850 python3 -u tests/tools/full_frame_check.py --grid 500 --width 3840 --height 2160 --spp 1000 --block 46 --rows-from 1050 --rows-to 2160 > gpurun_out/r06_b/full_c5b.log 2>&1
