#!/bin/bash
# Match-only library variant: tools/mkmatch.sh NAME [-DFLAG=V ...] -> variants/match_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -shared "$@" \
  -I "$R/include" "$R/mast3r-slam-ysh_amd/csrc/m3s_match.hip" -o "$R/variants/match_$name.so"
