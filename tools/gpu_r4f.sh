set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "subtree_factor or block_dataflow or sparse_llt_matches or broken_plan or tail_over or tail_pairs or over_capacity or pipelined_gathering or partial_trip" -v -s --timeout 200 --timeout-method thread > $OUT/r4f_solver.log 2>&1 || { echo "solver tests failed"; grep -E "FAILED|Error|assert" $OUT/r4f_solver.log | head -20; tail -30 $OUT/r4f_solver.log; exit 1; }
tail -3 $OUT/r4f_solver.log
timeout -k 10 300 python -u tools/solve_ab.py > $OUT/r4f_solve_ab.txt 2>&1 || { echo "solve_ab failed"; tail -20 $OUT/r4f_solve_ab.txt; exit 1; }
cat $OUT/r4f_solve_ab.txt | grep -v amdgpu.ids
N=256 M3S_SUBTREE=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4f_stamps_new.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4f_stamps_new.txt; exit 1; }
cat $OUT/r4f_stamps_new.txt | grep -v amdgpu.ids
N=256 M3S_SUBTREE=0 M3S_TAIL_PAIR=0 timeout -k 10 200 python -u tools/col_stamps.py variants/lib_colst.so > $OUT/r4f_stamps_old.txt 2>&1 || { echo "stamps old failed"; tail -20 $OUT/r4f_stamps_old.txt; exit 1; }
cat $OUT/r4f_stamps_old.txt | grep -v amdgpu.ids
