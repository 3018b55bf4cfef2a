#!/bin/bash
# Round 5: bisect the dense-fallback step-2 pose error over library variants (M3S_LIB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5u
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
for v in vcur vnolin vnonorm vnone; do
  M3S_LIB=$R/variants/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread "tests/test_gpu_backend.py::test_gn_over_capacity_plan_takes_dense_fallback" > $OUT/$v.log 2>&1
  echo "$v rc=$?"; grep "dense fallback N=" $OUT/$v.log
done
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_pkw3.so variants/lib_pkw4.so variants/lib_pkw2.so > $OUT/ab_pkw.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_pkw.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_pkw.txt
