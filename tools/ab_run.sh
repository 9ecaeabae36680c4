L=gibson_amd
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "not serial" > gpurun_out/par.log 2>&1 ; tail -2 gpurun_out/par.log
timeout -k 10 200 python tools/ab_compress.py 1 4096 262144 5 $L/liblzf_hip_prev.so $L/liblzf_hip.so $EXTRA > gpurun_out/ab.log 2>&1 && timeout -k 10 200 python tools/ab_compress.py 2 65536 16384 3 $L/liblzf_hip_prev.so $L/liblzf_hip.so $EXTRA >> gpurun_out/ab.log 2>&1 && timeout -k 10 200 python tools/ab_compress.py 3 16384 65536 3 $L/liblzf_hip_prev.so $L/liblzf_hip.so $EXTRA >> gpurun_out/ab.log 2>&1
grep -v amdgpu.ids gpurun_out/ab.log | grep -v identical
grep -c "identical.*True" gpurun_out/ab.log
