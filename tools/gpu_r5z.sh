#!/bin/bash
# Round 5: tracker pixel pairs (parity + A/B), tail form_x split (parity + A/B vs HEAD).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5z
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_tracker.py tests/test_gpu_backend.py -k "tracker or track or tail or sparse_llt or workers or broken" > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/trk_ab.py variants/lib_tpp0.so variants/lib_tpp1.so > $OUT/trk_ab.txt 2>&1 || { echo "trk ab failed"; tail -20 $OUT/trk_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/trk_ab.txt
AB_CASES="calib:256:12:16:3:16:1003,calib:128:12:16:3:16:1003" AB_ROUNDS=9 timeout -k 10 400 python -u tools/ab_calls.py variants/lib_headA.so variants/lib_curA.so > $OUT/ab_calls.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
