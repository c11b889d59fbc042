# Wide softmax split tiles: linear GPU tests, then the shape bench under rocprof.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${R06_OUT:-r06s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "linear" > $O/pytest_linear.log 2>&1 || { grep -E "FAILED|Error|error" $O/pytest_linear.log | head -20; tail -30 $O/pytest_linear.log; exit 1; }
tail -1 $O/pytest_linear.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/r06/linear_split_bench.py > $O/linear_split.log 2>&1 || { tail -30 $O/linear_split.log; exit 1; }
find $O -name "*_trace.csv" -delete
grep '^{' $O/linear_split.log | grep -E "\"C\": (1000|512|300)"
