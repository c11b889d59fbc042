# xgb1000: the whole-ensemble kernel with each row's trees split over P
# workgroups (SCA_TREE_SPLIT=P) vs one workgroup: microbench (correctness and
# us per batch), tree GPU tests with the split on, serving kernel percentiles,
# REST A/B.
set -o pipefail
O=gpurun_out/r05sl
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python tools/tree_microbench.py --small --rows 1,9,32,128 --iters 300 > $O/small.jsonl 2> $O/small.err || { tail -20 $O/small.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05sl/small.jsonl"):
    d = json.loads(l)
    print(d["rows"], {k: (v["us"], v["max_err"], v.get("acc_rezeroed")) for k, v in d.items() if isinstance(v, dict) and (k.startswith("split") or k in ("whole_la21_tpt1",))})
PY
SCA_TREE_SPLIT=4 timeout -k 10 400 python -u -m pytest tests -m gpu -k "tree or xgb or forest or isolation or sklearn or lightgbm or bar_staged" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
for cfg in 0.host 4.host 8.host 4.bar 8.bar 0.bar; do
  sp=${cfg%.*}; mode=${cfg#*.}
  (cd /tmp && SCA_TREE_SPLIT=$sp SCA_BATCH_INPUT=$mode SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/$O/db_$cfg" -o run -- python "$R/bench.py" --model xgb1000 --steps 10 --warmup 3 --extras none > "$R/$O/prof_$cfg.log" 2>&1) || exit 1
  db=$(find "$R/$O/db_$cfg" -name '*.db' | head -1)
  echo "split=$sp $mode: $(python tools/rocpd_stats.py "$db" --csv $O/kstats_$cfg.csv | sed -n 2p)"
  rm -rf "$R/$O/db_$cfg"
done
