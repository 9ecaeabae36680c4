#!/bin/bash
# Diagnostic library variant: one HIP source (default lzf_lane.hip, or
# SRC=lzf_decompress.hip ...) rebuilt with extra defines, linked with the
# other objects of the normal build (make first).
# usage: [SRC=file.hip] tools/build_variant.sh NAME -DFLAG [...]   -> gibson_amd/liblzf_hip_NAME.so
set -e
name=$1; shift
src=${SRC:-lzf_lane.hip}
cd "$(dirname "$0")/../gibson_amd/csrc"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics -I. -I../../include"
$H "$@" -c "$src" -o build/var_$name.o
$H -shared -o ../liblzf_hip_$name.so build/var_$name.o $(ls build/*.o | grep -v -e "build/${EXCL:-${src%.hip}.o}" -e var_ -e stats_ -e diag_ -e lzf_serial.o)
echo built gibson_amd/liblzf_hip_$name.so
