#!/bin/bash
# Build a variant of libsacx with extra kernel defines for A/B runs (SACX_LIBPATH=<out>):
#   tools/build_variant.sh <name> "<-DSACX_...=... flags>"  -> tools/libvar/libsacx_<name>.so
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p tools/libvar
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Iinclude -Isac-expert_amd/csrc"
$H $F $flags -mllvm -amdgpu-kernarg-preload-count=4 -c -o tools/libvar/k_sac_$name.o sac-expert_amd/csrc/k_sac.hip
$H $F $flags -c -o tools/libvar/sacx_$name.o sac-expert_amd/csrc/sacx.cpp
$H $F $flags -c -o tools/libvar/mtj_$name.o sac-expert_amd/csrc/mt_jump.cpp
$H --offload-arch=gfx950 -shared -o tools/libvar/libsacx_$name.so tools/libvar/k_sac_$name.o tools/libvar/sacx_$name.o \
    tools/libvar/mtj_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f tools/libvar/k_sac_$name.o tools/libvar/sacx_$name.o tools/libvar/mtj_$name.o
echo tools/libvar/libsacx_$name.so
