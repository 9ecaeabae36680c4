cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in A E; do
  LZF_HIP_LIB=gibson_amd/liblzf_hip_$v.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv -d gpurun_out/occ_$v -o run -- python3 bench.py --no-cpu --steps 1 --warmup 0 --count 262144 > gpurun_out/occ_$v.log 2>&1 || exit 1
  python3 tools/pmc_table.py gpurun_out/occ_$v
done
