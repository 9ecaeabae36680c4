#!/bin/bash
# GPU iteration for the window generation (LZF_GPU_KERNEL=wtab): its parity
# tests, then per-kernel times of the text64k bench under rocprofv3.
# usage (GPU box, repo root): tools/wtab_iter.sh [pytest -k expr] [bench args]
set -o pipefail
k=${1:-wtab}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread -k "$k" \
    > gpurun_out/wt.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/wt.log | tail -40; [ $rc = 0 ] || exit 1
LZF_GPU_KERNEL=wtab bash tools/kstats.sh gpurun_out/ks_wtab "$@" || exit 1
tail -1 gpurun_out/ks_wtab.log
