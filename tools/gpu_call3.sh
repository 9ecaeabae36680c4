# free-literal path with ballot gating: A/B of (trips, minimum lanes) on the lane and record parses
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=gibson_amd
V="$L/liblzf_hip_l0.so $L/liblzf_hip_lm4.so $L/liblzf_hip.so $L/liblzf_hip_lm16.so"
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 3 $V > gpurun_out/ab3.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 3 $V >> gpurun_out/ab3.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 0 8192 524288 3 $V >> gpurun_out/ab3.log 2>&1 || exit 1
R="$L/liblzf_hip_r0.so $L/liblzf_hip_rm4.so $L/liblzf_hip.so $L/liblzf_hip_rm16.so"
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 3 $R >> gpurun_out/ab3.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 65536 65536 3 $R >> gpurun_out/ab3.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab3.log | grep -v identical; grep -c "identical.*True" gpurun_out/ab3.log; grep -c "identical.*False" gpurun_out/ab3.log || true
