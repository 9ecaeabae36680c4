# record parse: a second, memory-free pass of the state machine per iteration (K3_NMPASS), gated by K3_NMMIN lanes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03k
L=gibson_amd
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 3 $L/liblzf_hip_nm0.so $L/liblzf_hip.so $L/liblzf_hip_nm16.so $L/liblzf_hip_nm1.so > gpurun_out/r03k/ab10.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 65536 65536 3 $L/liblzf_hip_nm0.so $L/liblzf_hip.so $L/liblzf_hip_nm16.so $L/liblzf_hip_nm1.so >> gpurun_out/r03k/ab10.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab_compress.py 2 65536 262144 2 $L/liblzf_hip_nm0.so $L/liblzf_hip.so >> gpurun_out/r03k/ab10.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03k/ab10.log
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 3 $L/liblzf_hip_ln0.so $L/liblzf_hip.so $L/liblzf_hip_ln16.so > gpurun_out/r03k/ab10l.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 3 $L/liblzf_hip_ln0.so $L/liblzf_hip.so $L/liblzf_hip_ln16.so >> gpurun_out/r03k/ab10l.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 0 8192 524288 3 $L/liblzf_hip_ln0.so $L/liblzf_hip.so $L/liblzf_hip_ln16.so >> gpurun_out/r03k/ab10l.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03k/ab10l.log
