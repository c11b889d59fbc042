# Round-6 xgb tail: tile kernel tests, microbench by batch size, and the
# xgb1000 serving A/B (SCA_TREE_TILE_ROWS=0 = r05 kernels) with kernel stats.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06e}
R=$GRAFT_REPO_ROOT
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "tree" > $O/pytest_tree.log 2>&1 || { tail -60 $O/pytest_tree.log; exit 1; }
tail -1 $O/pytest_tree.log
timeout -k 10 300 python3 tools/tree_microbench.py --small --rows 16,32,33,48,64,96,128,192,256 --iters 200 > $O/tree_small.jsonl 2>&1 || { tail -20 $O/tree_small.jsonl; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/r06e/tree_small.jsonl"):
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    sel = {k: d[k]["us"] for k in d if isinstance(d[k], dict) and (k in ("split8", "tile", "whole_la21_tpt1", "whole_la21_tpt2"))}
    print(d["rows"], sel, "tile_err", d.get("tile", {}).get("max_err"))
PY
for T in 0 256; do
  (cd /tmp && SCA_TREE_TILE_ROWS=$T SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_t$T -o xgb --output-format csv -- python3 $R/bench.py --model xgb1000 --steps 10 --warmup 3 --extras none > $R/$O/xgb_t$T.log 2>&1) || { tail -30 $O/xgb_t$T.log; exit 1; }
  grep '^{' $O/xgb_t$T.log | tail -1 | cut -c1-260
  f=$(find $O/prof_t$T -name '*kernel_stats.csv' | head -1); cp "$f" $O/xgb_t${T}_kernel_stats.csv; cut -c1-160 $O/xgb_t${T}_kernel_stats.csv | head -5
  find $O/prof_t$T -name '*kernel_trace.csv' -delete
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_kernels_gpu.py -k "linear" > $O/pytest_linear.log 2>&1 || { tail -60 $O/pytest_linear.log; exit 1; }
tail -1 $O/pytest_linear.log
timeout -k 10 240 python3 tools/r06/linear_bench.py > $O/linear_bench.log 2>&1 || { tail -30 $O/linear_bench.log; exit 1; }
grep '"mfma"' $O/linear_bench.log
