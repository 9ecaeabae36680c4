# record parse block size (K3_THREADS 64 / 128 vs 256) at configs[2]'s 256K values and at 128K
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03r
L=gibson_amd
timeout -k 10 400 python tools/ab_compress.py 2 65536 262144 2 $L/liblzf_hip.so $L/liblzf_hip_t64.so > gpurun_out/r03r/ab16.log 2>&1 || exit 1
timeout -k 10 400 python tools/ab_compress.py 2 65536 262144 2 $L/liblzf_hip.so $L/liblzf_hip_t128.so >> gpurun_out/r03r/ab16.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 3 $L/liblzf_hip.so $L/liblzf_hip_t64.so $L/liblzf_hip_t128.so >> gpurun_out/r03r/ab16.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03r/ab16.log
