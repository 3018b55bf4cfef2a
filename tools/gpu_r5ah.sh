#!/bin/bash
# Round 5: packed trip without the per-lane end test / offset selects, and the
# finalize's M formed on 49 lanes under the partial loads — parity + A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5ah
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_sim3.py tests/test_gpu_large.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_head.so variants/lib_pk272.so > $OUT/ab_lin.txt 2>&1 || { echo "ab_lin failed"; tail -20 $OUT/ab_lin.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_lin.txt
AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16" timeout -k 10 300 python -u tools/ab_calls.py variants/lib_head.so variants/lib_pk272.so > $OUT/ab_calls.txt 2>&1 || { echo "ab_calls failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
