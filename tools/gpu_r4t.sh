set -o pipefail
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python -u tools/trk_stamps.py variants/lib_trkst.so > $OUT/r4t_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/r4t_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/r4t_stamps.txt
