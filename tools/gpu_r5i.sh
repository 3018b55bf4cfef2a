#!/bin/bash
# Round 5: worker poll interval (build variants) x worker count (knob) A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5i
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB="gcomb=1;gcomb_wg=128|gcomb=1;gcomb_wg=64|gcomb=1;gcomb_wg=32|gcomb=0"
for L in mast3r-slam-ysh_amd/mast3r_slam_backends/libm3s_gn_test.so variants/lib_gs8_test.so variants/lib_gs24_test.so; do
  echo "== $L"
  LIB=$L SOLVE_AB="$AB" SOLVE_N="128,256" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/ab_$(basename $L).txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_$(basename $L).txt; exit 1; }
  grep -v amdgpu.ids $OUT/ab_$(basename $L).txt
done
