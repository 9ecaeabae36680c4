# diagnostic: cost of the parses' output stores (16-byte stores skipped), and lane-parse site counts
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03g
L=gibson_amd
timeout -k 10 300 python tools/ab_compress.py 1 4096 1048576 3 $L/liblzf_hip.so $L/liblzf_hip_lns.so > gpurun_out/r03g/ab5.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 3 16384 262144 3 $L/liblzf_hip.so $L/liblzf_hip_lns.so >> gpurun_out/r03g/ab5.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_compress.py 2 65536 262144 2 $L/liblzf_hip.so $L/liblzf_hip_rns.so >> gpurun_out/r03g/ab5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03g/ab5.log | grep -v identical
timeout -k 10 120 python tools/k2_sites.py 1 0x5EED0002 4096 65536 > gpurun_out/r03g/sites_json4k.txt 2>&1 || exit 1
timeout -k 10 120 python tools/k2_sites.py 3 0x5EED0005 16384 65536 > gpurun_out/r03g/sites_mixed16k.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03g/sites_*.txt | grep -v " 0.0 per"
