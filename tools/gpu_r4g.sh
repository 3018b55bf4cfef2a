set -o pipefail
OUT=gpurun_out; mkdir -p $OUT


timeout -k 10 300 python -u -m pytest tests/test_gpu_backend.py -k "tail or block_dataflow or sparse_llt_matches or warmup" -x -q --timeout 200 --timeout-method thread > $OUT/r4g_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/r4g_tests.log; exit 1; }
tail -2 $OUT/r4g_tests.log
N=256 M3S_SUBTREE=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4g_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4g_stamps.txt; exit 1; }
grep -A80 "dense tail" $OUT/r4g_stamps.txt
N=256 M3S_SUBTREE=0 M3S_TAIL_PAIR=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4g_stamps_cyc.txt 2>&1 || { echo "stamps failed"; exit 1; }
grep -A24 "dense tail" $OUT/r4g_stamps_cyc.txt
