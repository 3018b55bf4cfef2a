#!/bin/bash
# GPU-box: rocprofv3 kernel statistics of the default bench command, the PMC
# passes of the linearize kernels (tools/pmc_bench.sh) summarised into
# pmc/linearize_c3.json (packed kernel + the gathering kernel under "gather"),
# then the bench line again (now carrying roofline.traffic). TAG names outputs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-final}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python $R/bench.py --no-cpu > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats run failed"; tail -5 $OUT/stats_bench.err; exit 1; }
cd $R
TAG=$TAG/pmc bash tools/pmc_bench.sh || exit 1
python3 tools/pmc_summary.py $OUT/pmc linearize_packed_kernel pmc/linearize_c3.json 32 || exit 1
python3 tools/pmc_summary.py $OUT/pmc linearize_gather_kernel pmc/linearize_c3.json 32 gather || exit 1
cp pmc/linearize_c3.json $OUT/
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
