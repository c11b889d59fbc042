# xgb1000 after the lookahead descent: tree GPU tests, REST bench (2 runs),
# and a kernel-trace of one bench run.
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 400 python -u -m pytest tests -m gpu -k "tree or xgb or forest or isolation or sklearn or lightgbm" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05x/pytest_tree.log 2>&1 || { tail -30 gpurun_out/r05x/pytest_tree.log; exit 1; }
tail -2 gpurun_out/r05x/pytest_tree.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --model xgb1000 --steps 20 --warmup 5 --extras none > gpurun_out/r05x/bench_xgb.$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/r05x/bench_xgb.$i.log | tail -1 | cut -c1-400
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r05x/prof" -o xgb --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --model xgb1000 --steps 10 --warmup 3 --extras none > "$GRAFT_REPO_ROOT/gpurun_out/r05x/prof.log" 2>&1
