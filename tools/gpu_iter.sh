timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc = 0 ] || exit 1
timeout -k 10 120 python tools/kw_phases.py 1 0x5EED0002 4096 262144 > gpurun_out/ph.log 2>&1 || exit 1
timeout -k 10 120 python tools/k2_sites.py 1 0x5EED0002 4096 65536 >> gpurun_out/ph.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ph.log | grep -v " 0.0 per"
bash tools/kstats.sh gpurun_out/ks1
