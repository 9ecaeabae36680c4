L=gibson_amd
timeout -k 10 200 python tools/ab_compress.py 2 65536 65536 3 $L/liblzf_hip_prev.so $L/liblzf_hip.so > gpurun_out/ab.log 2>&1 && timeout -k 10 200 python tools/ab_compress.py 0 8192 262144 3 $L/liblzf_hip_prev.so $L/liblzf_hip.so >> gpurun_out/ab.log 2>&1 && timeout -k 10 200 python tools/ab_compress.py 3 16384 131072 3 $L/liblzf_hip_prev.so $L/liblzf_hip.so >> gpurun_out/ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; tail -3 gpurun_out/gputest.log; exit $rc
