#!/bin/bash
# GPU-box: sparse-LLT phase timing (N=64,128,256) over dense-tail thresholds (M3S_DENSE_TAIL_MIN).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
: > $OUT/tailmin_ab.txt
for tm in ${TMS:-24 16 12 8}; do
  echo "== M3S_DENSE_TAIL_MIN=$tm" >> $OUT/tailmin_ab.txt
  M3S_DENSE_TAIL_MIN=$tm M3S_LIB=$R/variants/lib_TB.so NS=64,128,256 timeout -k 10 200 python tools/llt_timing.py >> $OUT/tailmin_ab.txt 2>&1 || { echo "fail $tm"; tail -20 $OUT/tailmin_ab.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/tailmin_ab.txt
