# Narrow MFMA linear variants (K slices x chunk group) + the linear GPU tests.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "linear" > $O/pytest_linear.log 2>&1 || { tail -60 $O/pytest_linear.log; exit 1; }
tail -1 $O/pytest_linear.log
timeout -k 10 240 python3 tools/r06/linear_split_bench.py > $O/linear_split.log 2>&1 || { tail -30 $O/linear_split.log; exit 1; }
grep '^{' $O/linear_split.log
timeout -k 10 240 python3 tools/r06/linear_bench.py > $O/linear_bench.log 2>&1 || { tail -30 $O/linear_bench.log; exit 1; }
grep '"mfma"' $O/linear_bench.log
