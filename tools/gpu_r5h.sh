#!/bin/bash
# Round 5: sparse back-substitution workers (gcomb) — parity subset, whole-call
# A/B, launch timelines with and without the workers at 256 KFs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${RUN:-r5h}
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "tail or sparse_llt or dataflow or subtree or workers or broken or singular" tests/test_gpu_large.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SOLVE_AB="gcomb=1|gcomb=0" SOLVE_N="128,256" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/solve_ab_gcomb.txt 2>&1 || { echo "solve ab failed"; tail -20 $OUT/solve_ab_gcomb.txt; exit 1; }
grep -v amdgpu.ids $OUT/solve_ab_gcomb.txt
for k in 1 0; do
  SOLVE_AB="gcomb=$k" TAG=${RUN:-r5h}/trace256_g$k bash tools/prof_solve_small.sh > $OUT/solve_trace256_g$k.txt 2>&1 || { echo "trace failed"; tail -20 $OUT/solve_trace256_g$k.txt; exit 1; }
  echo "gcomb=$k"; cat $OUT/solve_trace256_g$k.txt
done
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst_g.so > $OUT/colst_g.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/colst_g.txt; exit 1; }
grep -A 12 "sparse workers" $OUT/colst_g.txt; grep "back-substitution done" $OUT/colst_g.txt
