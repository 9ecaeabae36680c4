# decoder bound: producer alone (consumer output ablated) vs full, and CD_TIMING phase balance, Zipf 8 KiB and sentence 64 KiB
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03m2
L=gibson_amd
export AB_MODE=decompress
timeout -k 10 300 python tools/ab_compress.py 0 8192 1048576 5 $L/liblzf_hip.so $L/liblzf_hip_dabl.so > gpurun_out/r03m2/ab12.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 5 $L/liblzf_hip.so $L/liblzf_hip_dabl.so >> gpurun_out/r03m2/ab12.log 2>&1 || exit 1
unset AB_MODE
timeout -k 10 300 python tools/dec_tstat.py 0 8192 1048576 $L/liblzf_hip_dtime.so >> gpurun_out/r03m2/ab12.log 2>&1 || exit 1
timeout -k 10 300 python tools/dec_tstat.py 2 65536 131072 $L/liblzf_hip_dtime.so >> gpurun_out/r03m2/ab12.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03m2/ab12.log
