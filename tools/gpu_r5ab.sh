#!/bin/bash
# Round 5: sparse packed iterations (M3S_PK_SPARSE) — parity on the sparse build, A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ab
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_sp0.so variants/lib_sp1.so > $OUT/ab_lin.txt 2>&1 || { echo "ab lin failed"; tail -20 $OUT/ab_lin.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_lin.txt
M3S_LIB=$R/variants/lib_sp1.so timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_ate.py tests/test_gpu_large.py -k "not test_lib" > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_CASES="calib:32:512:512:10:16:1003,rays:32:512:512:10:16:1003" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_sp0.so variants/lib_sp1.so > $OUT/ab_calls.txt 2>&1 || { echo "ab calls failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
