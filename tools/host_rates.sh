#!/bin/bash
# PCIe-inclusive host-path rates: staged and registered, one
# device and the two-context plan; one JSON line per run into $1 (a dir)
set -e
out=${1:-gpurun_out/host}
mkdir -p $out
export LZF_GPU_HOST_THREADS=16
for w in "2 65536 65536 text64k" "1 4096 524288 json4k" "3 16384 131072 mixed16k"; do
  set -- $w
  timeout -k 10 240 python tools/host_path_bench.py $1 $2 $3 5 > $out/host_$4_staged.json
  timeout -k 10 240 python tools/host_path_bench.py $1 $2 $3 5 --register > $out/host_$4_reg.json
  timeout -k 10 240 python tools/host_path_bench.py $1 $2 $3 5 --register --devices 0,0 > $out/host_$4_reg_dev00.json
done
