#!/bin/bash
# Round 5: ||dx|| wave sums on permlane/DPP (parity), packed-kernel waves-per-SIMD A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5t
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_large.py tests/test_gpu_ate.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_pkw3.so variants/lib_pkw4.so variants/lib_pkw2.so > $OUT/ab_pkw.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_pkw.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_pkw.txt
