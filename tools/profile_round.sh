#!/bin/bash
# Round profile on the GPU box (run from the repo root):
#   1. bench.py (default workload, with the CPU baseline)  -> OUT/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command -> OUT/trace
#   3. separate --pmc passes FETCH_SIZE / WRITE_SIZE        -> OUT/pmc_*
# usage: tools/profile_round.sh OUT [extra bench args]
set -e
out=$1; shift
mkdir -p "$out"
timeout -k 10 600 python3 bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --no-cpu "$@" > "$out/trace.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
    python3 bench.py --no-cpu --steps 1 --warmup 0 "$@" > "$out/pmc_fetch.log" 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
    python3 bench.py --no-cpu --steps 1 --warmup 0 "$@" > "$out/pmc_write.log" 2>&1
echo done
