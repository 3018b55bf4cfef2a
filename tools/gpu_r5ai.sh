#!/bin/bash
# Round 5: A/B with more rounds — HEAD, finalize-only, finalize + peeled packed trip.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ai
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB_ROUNDS=15 timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_head.so variants/lib_fin.so variants/lib_pk272.so variants/lib_c25.so > $OUT/ab_lin.txt 2>&1 || { echo "ab_lin failed"; tail -20 $OUT/ab_lin.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_lin.txt
AB_ROUNDS=15 AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_head.so variants/lib_fin.so variants/lib_pk272.so variants/lib_c25.so > $OUT/ab_calls.txt 2>&1 || { echo "ab_calls failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
timeout -k 10 200 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/llt_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/llt_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/llt_stamps.txt | head -40
