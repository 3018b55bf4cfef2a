#!/bin/bash
# Round 5: floors of the final packed kernel (no math / no loads variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5am
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB_ROUNDS=11 timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_final.so variants/lib_floor_mem.so variants/lib_floor_cmp.so > $OUT/ab_floor.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_floor.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_floor.txt
