# Defaults check after the split kernel became the small-batch default: tree GPU
# tests, REST xgb1000 (split 8 vs off, host vs BAR rows) and iris (host vs BAR).
set -o pipefail
O=gpurun_out/r05sl2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -k "tree or xgb or forest or isolation or sklearn or lightgbm or bar_staged" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_tree.log 2>&1 || { tail -30 $O/pytest_tree.log; exit 1; }
tail -1 $O/pytest_tree.log
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --model ${MODEL} --steps 20 --warmup 5 --extras none > $O/bench_$name.log 2>&1 || exit 1
  python - $O/bench_$name.log $name <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"], d["self_check"].get("max_abs_err"))
PY
}
for i in 1 2; do
  MODEL=xgb1000 run xgb_split8_host.$i SCA_BATCH_INPUT=host
  MODEL=xgb1000 run xgb_split0_host.$i SCA_TREE_SPLIT=0 SCA_BATCH_INPUT=host
  MODEL=xgb1000 run xgb_split8_bar.$i SCA_BATCH_INPUT=bar
  MODEL=iris run iris_host.$i SCA_BATCH_INPUT=host
  MODEL=iris run iris_bar.$i SCA_BATCH_INPUT=bar
done
