set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_outliers.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_outliers.log 2>&1 || { tail -30 gpurun_out/pytest_outliers.log; exit 1; }
tail -3 gpurun_out/pytest_outliers.log
STEPS="maha maha_jac" bash tools/gpu_check.sh
