#!/bin/bash
# Instruction mix / occupancy counters of the lzf kernels of one command, one
# --pmc pass per counter set (GPU box, repo root):
#   tools/pmc_mix.sh OUT python3 bench.py --mode decompress ...
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- "$@" > $out.p$i.log 2>&1 || exit 1
done
python3 tools/pmc_table.py $out/p1 $out/p2 $out/p3
