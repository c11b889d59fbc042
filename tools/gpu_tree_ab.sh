set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_batcher_signal_gpu.py tests/test_kernels_gpu.py -p no:cacheprovider > gpurun_out/ab/pytest.log 2>&1 || exit $?
for i in 1 2; do for f in 0 1; do
  SCA_TREE_FUSED=$f timeout -k 10 200 python bench.py --model xgb1000 --step-requests 20000 --extras none > gpurun_out/ab/xgb_f${f}_$i.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"p99_ms": [0-9.]*\|launch_frac": [0-9.]*' gpurun_out/ab/xgb_f${f}_$i.log | head -3 | tr '\n' ' '; echo " fused=$f"
done; done
export TMPDIR=/tmp
SCA_TREE_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_f1 -o run --output-format csv -- python3 bench.py --model xgb1000 --steps 3 --warmup 1 --step-requests 10000 --extras none > gpurun_out/ab/prof_f1.log 2>&1
