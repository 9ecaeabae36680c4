#!/bin/bash
# A/B of library builds and env settings on the bench (GPU box, repo root):
#   tools/ab_bench.sh "LABEL:ENV=.. ENV=..:LIB" ...   (LIB relative to gibson_amd/, "-" = default)
for spec in "$@"; do
    IFS=: read -r label envs lib <<< "$spec"
    libenv=""; [ "$lib" != "-" ] && libenv="LZF_HIP_LIB=$PWD/gibson_amd/$lib"
    r=$(env $envs $libenv timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu 2>/dev/null) || exit 1
    echo "$label $(echo "$r" | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["roofline"]["per_kernel_ms"])')"
done
