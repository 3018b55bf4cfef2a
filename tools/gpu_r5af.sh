#!/bin/bash
# Round 5: the dense tail launched beside df_factor_kernel (tail_conc) — parity + A/B + weak emulation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5af
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_large.py tests/test_gpu_sharded.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SOLVE_AB="tail_conc=1|tail_conc=0" SOLVE_N="128,256" SOLVE_ROUNDS=12 timeout -k 10 300 python -u tools/solve_ab.py > $OUT/solve_ab.txt 2>&1 || { echo "solve ab failed"; tail -20 $OUT/solve_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/solve_ab.txt
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
grep "world 8" $OUT/weak_emul.txt
