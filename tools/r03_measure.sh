#!/bin/bash
# Round-3 measurements after the stream cand kernel (GPU box, repo root):
# bench lines of the BASELINE workloads whose route changed, with rocprof
# kernel stats.  usage: tools/r03_measure.sh OUTDIR
out=${1:-gpurun_out/r03m}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {   # name, bench args...
    local name=$1; shift
    echo "== $name $(date +%T)"
    timeout -k 10 400 python bench.py "$@" > "$out/bench_$name.json" 2> "$out/bench_$name.err" || return 1
    tail -1 "$out/bench_$name.json" | cut -c1-300
}
stats() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ks_$name" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu "$@" > "$out/ks_$name.log" 2>&1 || return 1
    python3 profiles/summarize.py "$out/ks_$name" "$*" > "$out/kernel_stats_$name.txt" 2>&1
    grep -E "lzf_(cand|parse|decomp)" "$out/kernel_stats_$name.txt"
}
run json4k --workload json4k && stats json4k --workload json4k &&
run mixed16k_4M --workload mixed16k --total 4194304 --steps 3 &&
stats mixed16k_4M --workload mixed16k --total 4194304 &&
run text8k_rt --workload text8k --steps 3 &&
run text64k && echo done
