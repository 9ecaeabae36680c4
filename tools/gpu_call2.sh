# free-literal fast path in the lane parse: GPU suite on the product build (K2_LITX=3), A/B against 0/1/7
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc = 0 ] || exit 1
L=gibson_amd
V="$L/liblzf_hip_l0.so $L/liblzf_hip_l1.so $L/liblzf_hip.so $L/liblzf_hip_l7.so"
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 3 $V > gpurun_out/ab2.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 3 $V >> gpurun_out/ab2.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 0 8192 524288 3 $V >> gpurun_out/ab2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab2.log
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 3 $L/liblzf_hip_r0.so $L/liblzf_hip.so $L/liblzf_hip_r7.so > gpurun_out/ab2r.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 65536 65536 3 $L/liblzf_hip_r0.so $L/liblzf_hip.so >> gpurun_out/ab2r.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab2r.log
