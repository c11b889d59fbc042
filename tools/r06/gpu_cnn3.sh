# CNN GPU tests + ensemble bench (components on their own streams).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06n6}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_cnn.py tests/test_examples.py > $O/pytest_cnn.log 2>&1 || { tail -40 $O/pytest_cnn.log; exit 1; }
tail -1 $O/pytest_cnn.log
timeout -k 10 300 python3 -u tools/r06/imagenet_bench.py > $O/ensemble.log 2>&1 || { tail -40 $O/ensemble.log; exit 1; }
grep '^{' $O/ensemble.log | cut -c1-300
