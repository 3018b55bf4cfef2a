#!/bin/bash
# Round 5: one-level tracker reduction (M3S_TRK_FLAT) — tracker tests + A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5q
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tracker.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_flat0.so variants/lib_flat1.so variants/lib_flat0.so variants/lib_flat1.so > $OUT/trk_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/trk_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/trk_ab.txt
