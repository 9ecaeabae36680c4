# record parse: 32-record (128-byte, whole-line) blocks vs 16 at configs[2]'s full 256 K values; GPU suite on the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03i
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i/t8.log 2>&1; rc=$?; tail -3 gpurun_out/r03i/t8.log; [ $rc = 0 ] || exit 1
L=gibson_amd
timeout -k 10 400 python tools/ab_compress.py 2 65536 262144 3 $L/liblzf_hip.so $L/liblzf_hip_cb32.so > gpurun_out/r03i/ab8.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 65536 65536 3 $L/liblzf_hip.so $L/liblzf_hip_cb32.so >> gpurun_out/r03i/ab8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03i/ab8.log
