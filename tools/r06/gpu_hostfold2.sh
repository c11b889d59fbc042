# Host-folded split batches: tree / graph GPU tests, then xgb1000 serving A/B
# (SCA_TREE_HOST_FOLD 1 vs 0) with kernel stats.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06j}
R=$GRAFT_REPO_ROOT
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py tests/test_device_graph.py tests/test_gpu_serving.py tests/test_batcher_signal_gpu.py tests/test_outliers.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for H in 1 0; do
  (cd /tmp && SCA_TREE_HOST_FOLD=$H SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_h$H -o xgb --output-format csv -- python3 $R/bench.py --model xgb1000 --steps 10 --warmup 3 --extras none > $R/$O/xgb_h$H.log 2>&1) || { tail -30 $O/xgb_h$H.log; exit 1; }
  grep '^{' $O/xgb_h$H.log | tail -1 | cut -c1-200
  f=$(find $O/prof_h$H -name '*kernel_stats.csv' | head -1); cp "$f" $O/xgb_h${H}_kernel_stats.csv
  find $O/prof_h$H -name '*kernel_trace.csv' -delete
  python3 - $O/xgb_h${H}_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "perfect" in r["Name"]]
calls = sum(int(r["Calls"]) for r in rows); tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    n = r["Name"]; i = n.find("perfect"); print(n[i:n.find("(", i)], r["Calls"], round(float(r["AverageNs"]) / 1000, 2))
print("mean over tree dispatches us", round(tot / calls / 1000, 3), "calls", calls)
PY
done
SCA_TREE_HOST_FOLD=1 timeout -k 10 300 python3 bench.py --model xgb1000 > $O/xgb_plain.log 2>&1 || { tail -30 $O/xgb_plain.log; exit 1; }
grep '^{' $O/xgb_plain.log | tail -1 | cut -c1-300
