#!/bin/bash
# GPU-box: GPU tests, then sparse-LLT phase timing with the tail border spread
# over the chip (border_kernel) and inside the one-workgroup kernel (A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
: > $OUT/border_ab.txt
for sp in 1 0; do
  echo "== M3S_BORDER_SPLIT=$sp" >> $OUT/border_ab.txt
  M3S_BORDER_SPLIT=$sp M3S_LIB=$R/variants/lib_TS.so NS=128,256 BT=1 timeout -k 10 200 python tools/llt_timing.py >> $OUT/border_ab.txt 2>&1 || { echo "fail $sp"; tail -20 $OUT/border_ab.txt; exit 1; }
done
cat $OUT/border_ab.txt
MODES=sparse timeout -k 10 300 python tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
cat $OUT/weak_emul.txt
