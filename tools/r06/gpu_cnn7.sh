# CNN GPU tests (ResNet tuned at 4 buckets) + ensemble with tuned models and a 4-worker transformer.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n10}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_cnn.py > $O/pytest_cnn.log 2>&1 || { tail -40 $O/pytest_cnn.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_cnn.log | tail -6
IMAGENET_TR_WORKERS=4 timeout -k 10 600 python3 -u tools/r06/imagenet_bench.py > $O/ensemble_w4.log 2>&1 || { tail -40 $O/ensemble_w4.log; exit 1; }
grep '^{' $O/ensemble_w4.log | cut -c1-250
