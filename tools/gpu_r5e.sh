#!/bin/bash
# Round 5: where the solves spend their time now: the 256-KF launch timeline
# (kernel trace), the 256-KF column stamps, the C3 LLT item stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5e
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
TAG=r5e/trace256 bash tools/prof_solve_small.sh > $OUT/solve_trace256.txt 2>&1 || { echo "trace failed"; tail -20 $OUT/solve_trace256.txt; exit 1; }
cat $OUT/solve_trace256.txt
N=256 timeout -k 10 300 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/col_stamps256.txt 2>&1 || { echo "col stamps failed"; tail -20 $OUT/col_stamps256.txt; exit 1; }
grep -v amdgpu.ids $OUT/col_stamps256.txt | head -60
timeout -k 10 300 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/llt_stamps_c3.txt 2>&1 || { echo "llt stamps failed"; tail -20 $OUT/llt_stamps_c3.txt; exit 1; }
grep -v amdgpu.ids $OUT/llt_stamps_c3.txt | head -12
