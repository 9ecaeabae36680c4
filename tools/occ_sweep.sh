#!/bin/bash
# Residency sweep of the lane kernels (run on the GPU box from the repo root):
# kernel time per setting of LZF_LANE_{DEC,PARSE}_BLOCKS (blocks per CU).
# usage: tools/occ_sweep.sh OUT [bench args]
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for bl in 0 1 2 3 4 6; do
    LZF_LANE_DEC_BLOCKS=$bl LZF_LANE_PARSE_BLOCKS=$bl timeout -k 10 200 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$out/b$bl" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu "$@" \
        > "$out/b$bl.log" 2>&1 || exit 1
    echo "blocks/CU=$bl"; grep -h "lzf_" "$out/b$bl/run_kernel_stats.csv" | cut -d, -f1,4 | grep -v synth
done
