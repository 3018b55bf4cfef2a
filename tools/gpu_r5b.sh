#!/bin/bash
# Round 5, second box: the changed parity tests, the refine_matches A/B, the
# whole GPU suite, smoke and a quick bench line. Any failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5b
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_backend.py::test_gn_over_capacity_plan_takes_dense_fallback" tests/test_gpu_matching.py > $OUT/new_tests.log 2>&1 \
  || { echo "new tests failed"; grep -E "dense fallback|FAILED|Error|assert" $OUT/new_tests.log | head -20; tail -30 $OUT/new_tests.log; exit 1; }
grep -E "dense fallback|passed|failed" $OUT/new_tests.log
timeout -k 10 300 python -u tools/refine_ab.py variants/match_v1.so variants/match_v2.so variants/match_v2noxcd.so > $OUT/refine_ab.txt 2>&1 || { echo "refine ab failed"; tail -20 $OUT/refine_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/refine_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
