#!/bin/bash
# Round 5: the tail back-substitution through Z = L^-1 (tail_zinv_col):
# its parity tests, C4/C5 ATE, the solve A/B, the weak-scaling emulation;
# refine row-order A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5d
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "tail or sparse_llt or large or dataflow" > $OUT/tail_tests.log 2>&1 \
  || { echo "tail tests failed"; grep -E "FAILED|Error|assert" $OUT/tail_tests.log | head -20; tail -30 $OUT/tail_tests.log; exit 1; }
tail -1 $OUT/tail_tests.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_large.py > $OUT/large_tests.log 2>&1 \
  || { echo "large tests failed"; grep -E "FAILED|Error|assert" $OUT/large_tests.log | head -20; tail -30 $OUT/large_tests.log; exit 1; }
grep -E "ATE|passed|failed" $OUT/large_tests.log | tail -12
SOLVE_AB="tail_zinv=1|tail_zinv=0" SOLVE_N="128,256" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/solve_ab_zinv.txt 2>&1 || { echo "solve ab failed"; tail -20 $OUT/solve_ab_zinv.txt; exit 1; }
grep -v amdgpu.ids $OUT/solve_ab_zinv.txt
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
grep -v amdgpu.ids $OUT/weak_emul.txt
timeout -k 10 300 python -u tools/refine_ab.py variants/match_v2.so variants/match_v2rows.so > $OUT/refine_ab.txt 2>&1 || { echo "refine ab failed"; tail -20 $OUT/refine_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/refine_ab.txt
