#!/bin/bash
# Instruction mix of the compress kernels for libraries given as arguments
# (GPU box, repo root): tools/pmc_parse.sh OUT KIND N COUNT LIB...
out=$1; kind=$2; n=$3; count=$4; shift 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do
    tag=$(basename $lib .so)
    i=0
    for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
               "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        LZF_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/$tag/p$i -o run -- \
            python3 tools/compress_once.py $kind $n $count > $out.$tag.p$i.log 2>&1 || exit 1
    done
    echo "== $tag"
    python3 tools/pmc_table.py $out/$tag/p1 $out/$tag/p2 | grep parse
done
