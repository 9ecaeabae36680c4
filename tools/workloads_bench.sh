#!/bin/bash
# bench.py line per workload, default settings (GPU box, repo root)
for w in "$@"; do
    r=$(timeout -k 10 400 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu 2>/dev/null) || exit 1
    echo "$w $(echo "$r" | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());c=d["config"];print(d["value"], "GB/s", d["roofline"]["per_kernel_ms"], "ratio", c["ratio"], "compressed", c["compressed_fraction"])')"
done
