#!/bin/bash
# Per-kernel times of one compress (tools/compress_once.py) per library
# (GPU box, repo root): tools/kstats_lib.sh OUT KIND N COUNT LIB...
out=$1; kind=$2; n=$3; count=$4; shift 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
    tag=$(basename $lib .so)
    LZF_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o run -- \
        python3 tools/compress_once.py $kind $n $count > $out.$tag.log 2>&1 || exit 1
    echo "== $tag"
    python3 profiles/summarize.py $out/$tag "$tag" | grep -E "lzf_" | grep -v synth
done
