#!/bin/bash
# Round 5: tail back-substitution permlane shuffles + worker 7-sum on DPP (parity + A/B vs HEAD),
# tracker 7x7 solve fp32 vs fp64 (A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5s
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "tail or sparse_llt or dataflow or subtree or workers or broken or singular" tests/test_gpu_large.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
AB_CASES="calib:256:12:16:3:16:1003,calib:128:12:16:3:16:1003,calib:32:512:512:10:16:1003" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_head.so variants/lib_new.so > $OUT/ab_calls.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_f64.so variants/lib_f32.so variants/lib_f64.so variants/lib_f32.so > $OUT/trk_ab.txt 2>&1 || { echo "trk ab failed"; tail -20 $OUT/trk_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/trk_ab.txt
