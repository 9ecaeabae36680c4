cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/calib2
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/calib2/trace -o run -- ./tools/fetch_calib_bin > /dev/null || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/calib2/trace/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Kernel_Name"].split("(")[0], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
PY
