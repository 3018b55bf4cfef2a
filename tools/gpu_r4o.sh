set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "tail or warmup or block_dataflow or large" -x -q --timeout 200 --timeout-method thread > $OUT/r4o_tail.log 2>&1 || { echo "tail tests failed"; tail -20 $OUT/r4o_tail.log; exit 1; }
tail -1 $OUT/r4o_tail.log
SOLVE_AB="tail_pair=1|tail_pair=0" timeout -k 10 300 python -u tools/solve_ab.py > $OUT/r4o_solve_ab.txt 2>&1 || { echo "solve_ab failed"; tail -20 $OUT/r4o_solve_ab.txt; exit 1; }
grep -v amdgpu $OUT/r4o_solve_ab.txt
N=256 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4o_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4o_stamps.txt; exit 1; }
grep -A30 "dense tail" $OUT/r4o_stamps.txt | head -30
