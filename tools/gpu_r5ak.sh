#!/bin/bash
# Round 5: gathering launch with 24-bit index products (no quarter-rate
# v_mul_lo_u32) — parity + A/B against the committed library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ak
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_large.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_ROUNDS=15 timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_c25.so variants/lib_g24.so variants/lib_llt24.so > $OUT/ab_lin.txt 2>&1 || { echo "ab_lin failed"; tail -20 $OUT/ab_lin.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_lin.txt
AB_ROUNDS=15 AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16,rays:128:64:64:3:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_c25.so variants/lib_g24.so variants/lib_llt24.so > $OUT/ab_calls.txt 2>&1 || { echo "ab_calls failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
