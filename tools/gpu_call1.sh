# round-3 re-entry: GPU suite, cache-policy A/Bs (nt loads in the parses, sc1 record stores), round-3 measurements
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc = 0 ] || exit 1
L=gibson_amd
timeout -k 10 300 python tools/ab_compress.py 2 65536 131072 3 $L/liblzf_hip.so $L/liblzf_hip_nt.so $L/liblzf_hip_sc1.so $L/liblzf_hip_ntsc1.so > gpurun_out/ab1.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 3 $L/liblzf_hip.so $L/liblzf_hip_lnt.so >> gpurun_out/ab1.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab1.log
bash tools/r03_measure.sh gpurun_out/r03m
