#!/bin/bash
# Round 5: confirmation A/Bs with rotated orders (tracker reductions, sparse back-substitution workers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5w
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_xred0.so variants/lib_xred1.so > $OUT/trk_ab.txt 2>&1 || { echo "trk ab failed"; tail -20 $OUT/trk_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/trk_ab.txt
SOLVE_AB="gcomb=1|gcomb=0" SOLVE_N="128,256" SOLVE_ROUNDS=12 timeout -k 10 300 python -u tools/solve_ab.py > $OUT/solve_ab.txt 2>&1 || { echo "solve ab failed"; tail -20 $OUT/solve_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/solve_ab.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_ate.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_CASES="calib:32:512:512:10:16:1003,calib:32:128:128:10:16:1003,rays:24:128:128:10:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_bs7.so variants/lib_bs49.so > $OUT/ab_bs49.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_bs49.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_bs49.txt
