# 64 KiB values at configs[2]'s full size: table generation (default) vs the lane generation (stream cand + lane parse)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03l
timeout -k 10 500 python tools/ab_env.py 2 65536 262144 2 '' 'LZF_GPU_KERNEL=lane' > gpurun_out/r03l/ab11.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_env.py 3 65536 65536 3 '' 'LZF_GPU_KERNEL=lane' >> gpurun_out/r03l/ab11.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03l/ab11.log
