#!/bin/bash
# Round 5: the sparse back-substitution on the tail launch's workers
# (gcol_worker): parity, whole-call A/B, 256-KF launch timeline, weak emulation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5g
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "tail or sparse_llt or dataflow or subtree or workers or broken or singular" tests/test_gpu_large.py tests/test_gpu_sharded.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SOLVE_AB="gcomb=1|gcomb=0" SOLVE_N="128,256" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/solve_ab_gcomb.txt 2>&1 || { echo "solve ab failed"; tail -20 $OUT/solve_ab_gcomb.txt; exit 1; }
grep -v amdgpu.ids $OUT/solve_ab_gcomb.txt
SOLVE_AB="gcomb=1" TAG=r5g/trace256 bash tools/prof_solve_small.sh > $OUT/solve_trace256.txt 2>&1 || { echo "trace failed"; tail -20 $OUT/solve_trace256.txt; exit 1; }
cat $OUT/solve_trace256.txt
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
grep -v amdgpu.ids $OUT/weak_emul.txt
