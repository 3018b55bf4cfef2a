#!/bin/bash
# GPU-box: GPU tests, then sparse-LLT phase timing (N=128, 256) of the
# variants/lib_T<tag>.so builds listed in TAGS (-DM3S_LLT_TIMING=1 builds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
: > $OUT/tail_ab.txt
for s in ${TAGS:-8 22 41}; do
  echo "== variant T$s" >> $OUT/tail_ab.txt
  M3S_LIB=$R/variants/lib_T$s.so NS=128,256 BT=1 timeout -k 10 200 python tools/llt_timing.py >> $OUT/tail_ab.txt 2>&1 || { echo "fail $s"; tail -20 $OUT/tail_ab.txt; exit 1; }
done
cat $OUT/tail_ab.txt
