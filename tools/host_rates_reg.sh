#!/bin/bash
# registered-arena host-path rates only (one device), JSON lines into $1
set -e
out=${1:-gpurun_out/host}
mkdir -p $out
for w in "2 65536 65536 text64k" "1 4096 524288 json4k" "3 16384 131072 mixed16k"; do
  set -- $w
  timeout -k 10 240 python tools/host_path_bench.py $1 $2 $3 5 --register > $out/host_$4_reg.json
done
