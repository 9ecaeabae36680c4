#!/bin/bash
# Decode-path profile on the GPU box (repo root): BASELINE configs[3]
# (8 M x 8 KiB pre-compressed blocks), bench line + rocprofv3 kernel stats
# + FETCH/WRITE PMC passes.   usage: tools/decode_round.sh OUT
set -e
out=$1; shift
mkdir -p "$out"
timeout -k 10 300 python3 bench.py --mode decompress "$@" > "$out/bench.json" 2> "$out/bench.err"
cat "$out/bench.json"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 bench.py --mode decompress --no-cpu "$@" > "$out/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- \
    python3 bench.py --mode decompress --no-cpu --steps 1 --warmup 0 "$@" > "$out/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- \
    python3 bench.py --mode decompress --no-cpu --steps 1 --warmup 0 "$@" > "$out/pmc_write.log" 2>&1
echo done
