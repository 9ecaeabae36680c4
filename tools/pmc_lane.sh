#!/bin/bash
# Instruction-mix and LDS counters of the lane kernels, one --pmc pass per set
# (GPU box, repo root): tools/pmc_lane.sh OUT
out=${1:-gpurun_out/pmc_lane}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- \
        python3 bench.py --no-cpu --steps 1 --warmup 0 > $out.p$i.log 2>&1 || exit 1
done
python3 tools/pmc_table.py $out/p1 $out/p2
