#!/bin/bash
# GPU-box: the -m gpu tests, smoke(), the weak-scaling emulation and the
# default bench line. Each GPU step has its own time limit; any failure ends
# the script. TAG names the outputs; SKIP_TESTS=1 / SKIP_EMUL=1 / SKIP_BENCH=1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${TAG:-run}
mkdir -p $OUT
cd $R
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 900 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/${TAG}_gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $OUT/${TAG}_gpu_tests.log | head -20; tail -5 $OUT/${TAG}_gpu_tests.log; exit 1; }
tail -1 $OUT/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/${TAG}_smoke.log; exit 1; }
tail -1 $OUT/${TAG}_smoke.log
fi
if [ -z "${SKIP_EMUL:-}" ]; then
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/${TAG}_weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/${TAG}_weak_emul.txt; exit 1; }
cat $OUT/${TAG}_weak_emul.txt | grep -v amdgpu.ids
fi
if [ -z "${SKIP_BENCH:-}" ]; then
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -20 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
fi
