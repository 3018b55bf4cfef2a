#!/bin/bash
# GPU-box: rocprofv3 kernel trace of a short bench run at KF keyframes
# (MODE rays|calib) + a per-launch breakdown of one solve iteration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python $R/bench.py --kf-per-gpu ${KF:-256} --mode ${MODE:-rays} --steps 3 --warmup 1 --cold-steps 0 --no-cpu --no-tracker > $OUT/bench.json 2> $OUT/bench.err || { echo "profile failed"; tail -5 $OUT/bench.err; exit 1; }
python3 $R/tools/kernel_breakdown.py $OUT/run_kernel_trace.csv
