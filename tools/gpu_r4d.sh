set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "subtree_factor or block_dataflow or sparse_llt_matches or broken_plan or tail_over or tail_pairs" -v -s --timeout 200 --timeout-method thread > $OUT/r4d_solver.log 2>&1 || { echo "solver tests failed"; grep -E "FAILED|Error|assert" $OUT/r4d_solver.log | head -20; tail -30 $OUT/r4d_solver.log; exit 1; }
tail -3 $OUT/r4d_solver.log
timeout -k 10 300 python -u tools/solve_ab.py > $OUT/r4d_solve_ab.txt 2>&1 || { echo "solve_ab failed"; tail -20 $OUT/r4d_solve_ab.txt; exit 1; }
cat $OUT/r4d_solve_ab.txt | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SOLVE_N=256 SOLVE_ROUNDS=4 SOLVE_AB="subtree=1" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/r4d_prof -o r4d --output-format csv -- python3 tools/solve_ab.py > $OUT/r4d_prof.log 2>&1 || { echo "prof failed"; tail -20 $OUT/r4d_prof.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_backend.py -k "partial_trip or tiled or over_capacity or singular" -v -s --timeout 300 --timeout-method thread > $OUT/r4d_backend.log 2>&1 || { echo "backend tests failed"; tail -30 $OUT/r4d_backend.log; exit 1; }
tail -2 $OUT/r4d_backend.log
timeout -k 10 300 python bench.py --no-cpu --steps 10 > $OUT/r4d_bench.json 2> $OUT/r4d_bench.err || { echo "bench failed"; tail -30 $OUT/r4d_bench.err; exit 1; }
cat $OUT/r4d_bench.json
