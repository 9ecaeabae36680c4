# configs[4] (4M x 16 KiB mixed entropy, N=1, chunked) rocprof kernel stats after the free-literal path
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03q
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q/ks_mixed16k_4M -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --workload mixed16k --total 4194304 > gpurun_out/r03q/ks.log 2>&1 || exit 1
python3 profiles/summarize.py gpurun_out/r03q/ks_mixed16k_4M "bench.py --workload mixed16k --total 4194304 (round-3 final)" > gpurun_out/r03q/kernel_stats_mixed16k_4M_final.txt
grep -E "lzf_(cand|parse|decomp)" gpurun_out/r03q/kernel_stats_mixed16k_4M_final.txt
