set -o pipefail
mkdir -p gpurun_out/r06_full
timeout -k 10 300 python3 -u tests/tools/full_frame_check.py > gpurun_out/r06_full/full_c2.log 2>&1 &&
timeout -k 10 900 python3 -u tests/tools/full_frame_check.py --grid 500 --width 3840 --height 2160 --spp 1000 --block 46 --rows-from 0 --rows-to 1050 > gpurun_out/r06_full/full_c5a.log 2>&1
