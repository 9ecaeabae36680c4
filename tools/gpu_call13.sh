# decoder producer on aligned windows with the next window's jump tables built during ranking (CD_AHEAD): GPU suite, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03n
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03n/t13.log 2>&1; rc=$?; tail -3 gpurun_out/r03n/t13.log; [ $rc = 0 ] || exit 1
L=gibson_amd
export AB_MODE=decompress
timeout -k 10 300 python tools/ab_compress.py 0 8192 1048576 5 $L/liblzf_hip_dold.so $L/liblzf_hip.so > gpurun_out/r03n/ab13.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 5 $L/liblzf_hip_dold.so $L/liblzf_hip.so >> gpurun_out/r03n/ab13.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 5 $L/liblzf_hip_dold.so $L/liblzf_hip.so >> gpurun_out/r03n/ab13.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03n/ab13.log
