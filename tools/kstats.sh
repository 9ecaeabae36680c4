#!/bin/bash
# Per-kernel times of the lane kernels without the two-stream overlap
# (LZF_GPU_LANE_PIPE=0), one rocprofv3 --kernel-trace --stats run.
# usage (on the GPU box, repo root): tools/kstats.sh OUT [bench args]
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
LZF_GPU_LANE_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu "$@" > "$out.log" 2>&1 || exit 1
python3 profiles/summarize.py "$out" "$*" | grep -E "lzf_(cand|parse|wparse|decomp|compress|dec_)" | grep -v synth
