# lane parse free-literal gating for the lane-route BASELINE configs (json4k = configs[1], mixed16k = configs[4])
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03j
L=gibson_amd
V="$L/liblzf_hip_l0.so $L/liblzf_hip.so $L/liblzf_hip_l1u.so $L/liblzf_hip_lu1x2.so $L/liblzf_hip_lu1.so"
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 5 $V > gpurun_out/r03j/ab9.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 5 $V >> gpurun_out/r03j/ab9.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03j/ab9.log | grep -v identical; grep -c "identical.*True" gpurun_out/r03j/ab9.log
