#!/bin/bash
# Compress/decompress kernel times per workload for a few env settings (GPU box, repo root)
for w in "$@"; do
  for spec in "default:" "lanemid:LZF_GPU_LANE_MID=1"; do
    IFS=: read -r label envs <<< "$spec"
    r=$(env $envs timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu 2>/dev/null) || exit 1
    echo "$w $label $(echo "$r" | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["roofline"]["per_kernel_ms"])')"
  done
done
