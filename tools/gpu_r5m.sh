#!/bin/bash
# Round 5: gathering launch task order (KF j / KF i) and an identity-gather bound: time + fabric bytes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5m
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_ordj.so variants/lib_ordi.so variants/lib_ident.so > $OUT/ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab.txt
TAG=r5m/pmc bash tools/pmc_variants.sh variants/lib_ordj.so variants/lib_ordi.so variants/lib_ident.so
