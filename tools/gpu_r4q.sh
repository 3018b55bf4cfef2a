set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_large.py -x -q --timeout 400 --timeout-method thread > $OUT/r4q_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/r4q_tests.log | head; tail -20 $OUT/r4q_tests.log; exit 1; }
tail -1 $OUT/r4q_tests.log
AB_CASES="calib:256:12:16:3:16,rays:256:12:16:3:16,calib:128:12:16:3:16,calib:32:128:128:10:16" timeout -k 10 500 python -u tools/ab_calls.py variants/lib_before.so variants/lib_after.so > $OUT/r4q_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4q_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4q_ab.txt | tail -8
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4q_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4q_stamps.txt; exit 1; }
head -14 $OUT/r4q_stamps.txt | grep -v amdgpu
