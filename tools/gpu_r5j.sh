#!/bin/bash
# Round 5: workers at their defaults (64 workgroups, poll interval 8): stamps, weak emulation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5j
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst_g.so > $OUT/colst_g.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/colst_g.txt; exit 1; }
grep -A 12 "sparse workers" $OUT/colst_g.txt; grep "back-substitution done\|flags seen" $OUT/colst_g.txt
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
grep -v amdgpu.ids $OUT/weak_emul.txt
