# lane parse: two extension pieces per iteration for long matches, ballot-gated (K2_EXT2 lanes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03s
L=gibson_amd
V="$L/liblzf_hip.so $L/liblzf_hip_e8.so $L/liblzf_hip_e2.so"
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 5 $V > gpurun_out/r03s/ab17.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 5 $V >> gpurun_out/r03s/ab17.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 0 8192 524288 5 $V >> gpurun_out/r03s/ab17.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03s/ab17.log
