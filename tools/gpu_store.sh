set -u
OUT=${1:-gpurun_out/store}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 400 python -u tools/bench_e2e.py --size 1024 --radius 2 --repeat 2 > $OUT/e2e_bytes.txt 2>&1 || { echo "e2e rc=$?"; tail -20 $OUT/e2e_bytes.txt; exit 1; }
tail -1 $OUT/e2e_bytes.txt
timeout -k 10 400 python -u tools/bench_e2e.py --size 1024 --radius 2 --repeat 1 --codec gzip --check 0 > $OUT/e2e_gzip.txt 2>&1 || { echo "e2e gzip rc=$?"; tail -20 $OUT/e2e_gzip.txt; exit 1; }
tail -1 $OUT/e2e_gzip.txt
