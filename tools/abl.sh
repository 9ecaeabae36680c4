#!/bin/bash
# Ablation timing: per-kernel times for each diagnostic library build
# (results are NOT bit-exact for ablated builds: timing only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abl
for lib in "$@"; do
    echo "== $lib"
    LZF_HIP_LIB=$PWD/gibson_amd/$lib LZF_GPU_LANE_PIPE=0 env $ABL_ENV timeout -k 10 200 rocprofv3 --kernel-trace --stats \
        --output-format csv -d gpurun_out/abl/$lib -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu \
        > gpurun_out/abl/$lib.log 2>&1 || exit 1
    python3 profiles/summarize.py gpurun_out/abl/$lib x | grep -E "lzf_(cand|parse|decomp)"
done
