set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/maha_bench.py --p 20 --requests 1200 --threads 16 > gpurun_out/maha_dbg.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/maha_dbg.log
cat gpurun_out/maha_dbg.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_outliers.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_outliers.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_outliers.log
exit $rc
