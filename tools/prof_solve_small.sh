#!/bin/bash
# GPU-box: rocprofv3 kernel trace of tools/solve_ab.py (small images: the
# call is the solve) at SOLVE_N keyframes, then the launch timeline of the
# solve iterations (tools/solve_trace.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-solvetrace}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
SOLVE_AB="${SOLVE_AB:-tail_pair=1}" SOLVE_N="${SOLVE_N:-256}" SOLVE_ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $R/tools/solve_ab.py > $OUT/solve_ab.txt 2>&1 || { echo "trace failed"; tail -5 $OUT/solve_ab.txt; exit 1; }
f=$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/solve_trace.py $f
