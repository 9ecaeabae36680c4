#!/bin/bash
# Decoder A/B on three value shapes (GPU box, repo root): tools/ab_dec.sh LIB...
for w in "0 8192 1048576" "1 4096 1048576" "0 65536 131072"; do
  AB_MODE=decompress timeout -k 10 200 python tools/ab_compress.py $w 5 "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
