# end-of-round-3 profiles after the free-literal path and the decoder's wide stores:
# bench + rocprof stats + FETCH/WRITE passes for text64k (configs[2]), json4k (configs[1]), decode-only configs[3]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh gpurun_out/r03p/text64k || exit 1
tail -1 gpurun_out/r03p/text64k/bench.json | cut -c1-300
bash tools/profile_round.sh gpurun_out/r03p/json4k --workload json4k || exit 1
tail -1 gpurun_out/r03p/json4k/bench.json | cut -c1-300
bash tools/profile_round.sh gpurun_out/r03p/text8k_decode --mode decompress || exit 1
tail -1 gpurun_out/r03p/text8k_decode/bench.json | cut -c1-300
