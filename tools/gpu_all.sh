#!/bin/bash
# Whole GPU suite + smoke (GPU box, repo root): tools/gpu_all.sh [pytest -k expr]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
k=${1:+-k "$1"}
eval timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $k > gpurun_out/all.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|SKIP" gpurun_out/all.log | tail -12; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | grep -v amdgpu.ids
