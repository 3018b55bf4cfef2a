#!/bin/bash
# GPU-box: parity tests, bench (no CPU leg). Any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench_q.json 2> $OUT/bench_q.err || { echo "bench failed"; tail -30 $OUT/bench_q.err; exit 1; }
cat $OUT/bench_q.json
