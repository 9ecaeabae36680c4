#!/bin/bash
# FETCH_SIZE calibration run (GPU box, repo root): tools/fetch_calib.hip
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run -- ./tools/fetch_calib_bin || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/write -o run -- ./tools/fetch_calib_bin || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/calib/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Kernel_Name"].split("(")[0], r["Counter_Name"], r["Counter_Value"])
PY
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/calib/trace -o run -- ./tools/fetch_calib_bin > /dev/null || exit 1
python3 profiles/summarize.py gpurun_out/calib/trace calib | grep -E "16"
