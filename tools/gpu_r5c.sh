#!/bin/bash
# Round 5: changed parity tests (dense fallback, matching, tracker), the
# refine / tracker / gathering-grid A/Bs, the whole GPU suite, smoke, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5c
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_backend.py::test_gn_over_capacity_plan_takes_dense_fallback" tests/test_gpu_matching.py tests/test_gpu_tracker.py > $OUT/new_tests.log 2>&1 \
  || { echo "new tests failed"; grep -E "dense fallback|FAILED|Error|assert" $OUT/new_tests.log | head -20; tail -30 $OUT/new_tests.log; exit 1; }
grep -E "dense fallback|passed|failed" $OUT/new_tests.log
timeout -k 10 300 python -u tools/refine_ab.py variants/match_v1.so variants/match_v2.so variants/match_v2noxcd.so > $OUT/refine_ab.txt 2>&1 || { echo "refine ab failed"; tail -20 $OUT/refine_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/refine_ab.txt
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_trk_rec.so variants/lib_trk_topall.so variants/lib_trk_topall_ns.so > $OUT/trk_ab.txt 2>&1 || { echo "trk ab failed"; tail -20 $OUT/trk_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/trk_ab.txt
timeout -k 10 300 python -u tools/ab_linearize.py variants/lib_g6400.so variants/lib_g12800.so variants/lib_g25600.so variants/lib_g3200.so > $OUT/gather_ab.txt 2>&1 || { echo "gather ab failed"; tail -20 $OUT/gather_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/gather_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
