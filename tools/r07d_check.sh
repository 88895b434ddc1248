set -uo pipefail
OUT=gpurun_out/check_r07d; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --config 4 --no-cpu > $OUT/config4.json 2> $OUT/config4.err || { echo "bench4 failed"; tail -20 $OUT/config4.err; exit 1; }
cat $OUT/config4.json
