set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x --timeout 500 > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/ab_schedule.py --rounds 5 --libs new=raytracing-practice_amd/lib/librtgpu.so,ns=raytracing-practice_amd/lib/librtgpu_ns.so --variants ns@0:0:0,new@0:0:0,ns@0:0:0#0.7:4,new@0:0:0#0.7:4,new@0:0:0#0.5:8,new@0:0:0#0.3:1,new@0:40:0#0.7:4,new@0:56:0#0.7:4,new@0:0:8#0.7:4,new@0:0:16#0.7:4 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 3
