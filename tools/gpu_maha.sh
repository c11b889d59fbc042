set -o pipefail
mkdir -p gpurun_out
for p in 9 20 32 64; do timeout -k 5 60 ./tools/micro/jacobi_probe $p >> gpurun_out/jacobi_probe.txt 2>&1 || exit 1; done
cat gpurun_out/jacobi_probe.txt
timeout -k 10 400 python -u -m pytest tests/test_outliers.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_outliers.log 2>&1 || { tail -30 gpurun_out/pytest_outliers.log; exit 1; }
tail -3 gpurun_out/pytest_outliers.log
STEPS="maha maha_jac maha_hh" bash tools/gpu_check.sh
