#!/bin/bash
# GPU-box script: parity tests, bench, rocprofv3 kernel stats. Each GPU step
# has its own time limit; any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" && timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench failed"; tail -30 $OUT/bench1.err; exit 1; }
cat $OUT/bench1.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof1 -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 1 --no-cpu --no-tracker > $OUT/prof1_bench.json 2> $OUT/prof1.err || { echo "rocprof failed"; tail -30 $OUT/prof1.err; exit 1; }
find $OUT/prof1 -name "*stats*" | head
cd $R
MODES=sparse timeout -k 10 300 python tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
cat $OUT/weak_emul.txt
