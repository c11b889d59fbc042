set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_outliers.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_outliers.log 2>&1 || { tail -30 gpurun_out/pytest_outliers.log; exit 1; }
tail -2 gpurun_out/pytest_outliers.log
timeout -k 10 200 python -u tools/maha_bench.py --p 9 32 64 --requests 1000 --threads 16 --out gpurun_out/maha_phase.json > gpurun_out/maha_phase.log 2>&1
rc=$?; tail -4 gpurun_out/maha_phase.log; exit $rc
