#!/bin/bash
# Round 5 final evidence of the last library: rocprofv3 stats + PMC + bench
# with traffic (tools/final_prof.sh), then the weak-scaling emulation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=${TAG:-final_r5b} bash tools/final_prof.sh || exit 1
timeout -k 10 500 python -u tools/weak_emul.py > $R/gpurun_out/${TAG:-final_r5b}/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $R/gpurun_out/${TAG:-final_r5b}/weak_emul.txt; exit 1; }
grep "world" $R/gpurun_out/${TAG:-final_r5b}/weak_emul.txt | tail -8
