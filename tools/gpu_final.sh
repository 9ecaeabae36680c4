# final round-3 check of the committed tree: GPU suite, smoke, default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/t.log 2>&1; rc=$?; tail -3 gpurun_out/final/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/final/smoke.log | tail -3
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
tail -1 gpurun_out/final/bench.json | cut -c1-700
