set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_backend.py tests/test_gpu_large.py -x -q --timeout 400 --timeout-method thread > $OUT/r4r_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/r4r_tests.log | head; tail -20 $OUT/r4r_tests.log; exit 1; }
tail -1 $OUT/r4r_tests.log
AB_CASES="calib:256:12:16:3:16,rays:256:12:16:3:16,calib:128:12:16:3:16" timeout -k 10 500 python -u tools/ab_calls.py variants/lib_before.so variants/lib_after.so variants/lib_after2.so > $OUT/r4r_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r4r_ab.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4r_ab.txt | tail -9
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4r_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4r_stamps.txt; exit 1; }
grep -A22 "dense tail" $OUT/r4r_stamps.txt | head -22
