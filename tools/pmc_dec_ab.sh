#!/bin/bash
# Instruction-mix PMC of the decoder in several library builds (GPU box, repo
# root): tools/pmc_dec_ab.sh NAME...  (gibson_amd/liblzf_hip_NAME.so; "" = product)
set -e
for L in "$@"; do
  f=gibson_amd/liblzf_hip${L:+_$L}.so
  LZF_HIP_LIB=$PWD/$f bash tools/pmc_mix.sh gpurun_out/mix_$L python3 bench.py --mode decompress --count 1048576 --no-cpu --steps 1 --warmup 0 > gpurun_out/mix_$L.txt 2>&1
  echo "== $f"; grep decompress gpurun_out/mix_$L.txt
done
