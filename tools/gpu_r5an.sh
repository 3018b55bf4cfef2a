#!/bin/bash
# Round 5: packed-kernel grid target re-swept after the VALU cut.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5an
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB_ROUNDS=11 timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_final.so variants/lib_tb1536.so variants/lib_tb2560.so variants/lib_tb3072.so > $OUT/ab_tb.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_tb.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_tb.txt
AB_ROUNDS=9 AB_CASES="calib:32:512:512:10:16:1003" timeout -k 10 300 python -u tools/ab_calls.py variants/lib_final.so variants/lib_tb1536.so variants/lib_tb2560.so variants/lib_tb3072.so > $OUT/ab_calls_tb.txt 2>&1 || { echo "ab_calls failed"; tail -20 $OUT/ab_calls_tb.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls_tb.txt
