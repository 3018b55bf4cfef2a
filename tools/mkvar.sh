#!/bin/bash
# Build a library variant of the current tree: tools/mkvar.sh NAME [-DFLAG=V ...]
# -> variants/lib_NAME.so (git-ignored; shipped to the GPU box by gpurun).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/variants"
C="$R/mast3r-slam-ysh_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -shared "$@" \
  -I "$R/include" "$C/m3s_gn.hip" "$C/m3s_match.hip" "$C/m3s_fuse.hip" "$C/m3s_symbolic.cpp" \
  -o "$R/variants/lib_$name.so"
