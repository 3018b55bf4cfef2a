#!/bin/bash
# Round 5: border tasks waited per batch + batched col_finish loads: parity
# (bitwise vs the previous build, large-graph tests), whole-call A/B, the
# 256-KF launch timeline, weak-scaling emulation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5f
mkdir -p $OUT
cd $R
echo "torch import"; timeout -k 10 300 python -c "import torch; print(torch.cuda.is_available())" || exit 1
AB_CASES="calib:256:12:16:3:16,rays:256:12:16:3:16,rays:140:24:32:3:8,calib:128:12:16:3:16,calib:32:128:128:10:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_base_test.so mast3r-slam-ysh_amd/mast3r_slam_backends/libm3s_gn_test.so > $OUT/ab_calls.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_calls.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_calls.txt
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_backend.py -k "tail or sparse_llt or dataflow or subtree" tests/test_gpu_large.py > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
TAG=r5f/trace256 bash tools/prof_solve_small.sh > $OUT/solve_trace256.txt 2>&1 || { echo "trace failed"; tail -20 $OUT/solve_trace256.txt; exit 1; }
cat $OUT/solve_trace256.txt
timeout -k 10 600 python -u tools/weak_emul.py > $OUT/weak_emul.txt 2>&1 || { echo "weak_emul failed"; tail -20 $OUT/weak_emul.txt; exit 1; }
grep -v amdgpu.ids $OUT/weak_emul.txt
AB_CASES="calib:32:128:128:10:16,calib:32:512:512:10:16:1003,rays:24:64:64:10:16" timeout -k 10 400 python -u tools/ab_calls.py variants/lib_bs0.so mast3r-slam-ysh_amd/mast3r_slam_backends/libm3s_gn.so > $OUT/ab_bs_sync.txt 2>&1 || { echo "ab bs failed"; tail -20 $OUT/ab_bs_sync.txt; exit 1; }
grep -v amdgpu.ids $OUT/ab_bs_sync.txt
timeout -k 10 300 python -u tools/llt_stamps.py variants/lib_lst.so > $OUT/llt_stamps_c3.txt 2>&1 || { echo "llt stamps failed"; tail -20 $OUT/llt_stamps_c3.txt; exit 1; }
grep -v amdgpu.ids $OUT/llt_stamps_c3.txt | head -4
