# Round-6 A/Bs: split kernel with per-row-tile counters (microbench), the
# fused linear device graph (bench --graph pipeline, SCA_GRAPH_FUSE 1 / 0),
# and the HDP flush after BAR staging (xgb1000, SCA_HDP_FLUSH 1 / 0).
set -o pipefail
O=gpurun_out/${R06_OUT:-r06f}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "tree" > $O/pytest_tree.log 2>&1 || { tail -60 $O/pytest_tree.log; exit 1; }
tail -1 $O/pytest_tree.log
timeout -k 10 300 python3 tools/tree_microbench.py --small --rows 16,32,48,64,96,128,192,256 --iters 200 > $O/tree_small.jsonl 2>&1 || { tail -20 $O/tree_small.jsonl; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/r06f/tree_small.jsonl"):
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    sel = {k: d[k]["us"] for k in d if isinstance(d[k], dict) and (k.startswith("split") or k in ("tile", "whole_la21_tpt1", "whole_la21_tpt2"))}
    ok = all(d[k].get("acc_rezeroed", True) for k in d if isinstance(d[k], dict))
    print(d["rows"], sel, "rezeroed", ok)
PY
for F in 1 0; do
  SCA_GRAPH_FUSE=$F timeout -k 10 300 python3 bench.py --graph pipeline --extras none > $O/pipeline_fuse$F.log 2>&1 || { tail -30 $O/pipeline_fuse$F.log; exit 1; }
  grep '^{' $O/pipeline_fuse$F.log | tail -1 | cut -c1-300
done
for H in 1 0; do
  SCA_HDP_FLUSH=$H timeout -k 10 300 python3 bench.py --model xgb1000 --extras none > $O/xgb_hdp$H.log 2>&1 || { tail -30 $O/xgb_hdp$H.log; exit 1; }
  grep '^{' $O/xgb_hdp$H.log | tail -1 | cut -c1-300
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "linear" > $O/pytest_linear.log 2>&1 || { tail -60 $O/pytest_linear.log; exit 1; }
tail -1 $O/pytest_linear.log
timeout -k 10 240 python3 tools/r06/linear_bench.py > $O/linear_bench.log 2>&1 || { tail -30 $O/linear_bench.log; exit 1; }
grep '"mfma"' $O/linear_bench.log
