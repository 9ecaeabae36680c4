# GPU suite on the free-literal build; lane-parse site counts (json4k, mixed16k); configs[1] and configs[4] bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03f
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?; tail -3 gpurun_out/t4.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python tools/k2_sites.py 1 0x5EED0002 4096 65536 > gpurun_out/r03f/sites_json4k.txt 2>&1 || exit 1
timeout -k 10 120 python tools/k2_sites.py 3 0x5EED0005 16384 65536 > gpurun_out/r03f/sites_mixed16k.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r03f/sites_*.txt
timeout -k 10 400 python bench.py --workload mixed16k --total 4194304 --steps 3 > gpurun_out/r03f/bench_mixed16k_4M.json 2> gpurun_out/r03f/bench_mixed16k_4M.err || exit 1
tail -1 gpurun_out/r03f/bench_mixed16k_4M.json | cut -c1-400
timeout -k 10 400 python bench.py --workload json4k > gpurun_out/r03f/bench_json4k.json 2> gpurun_out/r03f/bench_json4k.err || exit 1
tail -1 gpurun_out/r03f/bench_json4k.json | cut -c1-400
