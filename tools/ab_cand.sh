#!/bin/bash
# cand-kernel only (LZF_GPU_TABLE_STAGE=1) A/B of library builds on text64k,
# then per-phase cycles from the -DKT_TIMING build.
# usage (GPU box, repo root): tools/ab_cand.sh LIB_A LIB_B [...]
export LZF_GPU_TABLE_STAGE=1
timeout -k 10 200 python tools/ab_compress.py 2 65536 65536 3 "$@" > gpurun_out/abc.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/abc.log | grep -v identical
timeout -k 10 120 python tools/kt_timing.py 2 65536 16384 > gpurun_out/ktt.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ktt.log
