# Round-6 split defaults A/B on xgb1000 serving: new (16 parts <= 16 rows,
# 8 parts to 96 rows) vs round-5 (8 parts to 32 rows), kernel stats each.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06h}
R=$GRAFT_REPO_ROOT
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "tree" > $O/pytest_tree.log 2>&1 || { tail -60 $O/pytest_tree.log; exit 1; }
tail -1 $O/pytest_tree.log
for cfg in new old; do
  if [ $cfg = old ]; then EXTRA="SCA_TREE_SPLIT=8 SCA_TREE_SPLIT_ROWS=32"; else EXTRA=""; fi
  (cd /tmp && env $EXTRA SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$cfg -o xgb --output-format csv -- python3 $R/bench.py --model xgb1000 --steps 10 --warmup 3 --extras none > $R/$O/xgb_$cfg.log 2>&1) || { tail -30 $O/xgb_$cfg.log; exit 1; }
  grep '^{' $O/xgb_$cfg.log | tail -1 | cut -c1-200
  f=$(find $O/prof_$cfg -name '*kernel_stats.csv' | head -1); cp "$f" $O/xgb_${cfg}_kernel_stats.csv
  find $O/prof_$cfg -name '*kernel_trace.csv' -delete
  python3 - $O/xgb_${cfg}_kernel_stats.csv <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "perfect" in r["Name"]]
calls = sum(int(r["Calls"]) for r in rows); tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    n = r["Name"]; i = n.find("perfect"); print(n[i:n.find("(", i)], r["Calls"], round(float(r["AverageNs"]) / 1000, 2))
print("mean over tree dispatches us", round(tot / calls / 1000, 3), "calls", calls)
PY
done
