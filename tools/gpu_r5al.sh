#!/bin/bash
# Round 5: PART items (pre-summed heads of long update lists) on the
# LDS-resident sparse_llt_kernel path — A/B + stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5al
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB_ROUNDS=11 AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16,rays:24:64:64:10:16,calib:48:64:64:10:16" timeout -k 10 500 python -u tools/ab_calls.py variants/lib_llt24.so variants/lib_split3.so variants/lib_split4.so variants/lib_split6.so > $OUT/ab_calls.txt 2>&1 || { echo "ab_calls failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
timeout -k 10 200 python -u tools/llt_stamps.py variants/lib_lstsplit4.so > $OUT/llt_stamps_split4.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/llt_stamps_split4.txt; exit 1; }
grep -v amdgpu.ids $OUT/llt_stamps_split4.txt | head -8
