# Round-6 microbenchmarks: hipGraph vs direct launches for K-kernel chains;
# tree kernels (whole vs split{4,8,16,32}) by batch size at xgb1000 shape.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06d}
mkdir -p $O
timeout -k 10 120 ./tools/micro/graph_cost > $O/graph_cost.jsonl 2>&1 || { cat $O/graph_cost.jsonl; exit 1; }
cat $O/graph_cost.jsonl
timeout -k 10 400 python3 tools/tree_microbench.py --small --rows 16,32,48,64,96,128,192 --iters 200 > $O/tree_small.jsonl 2>&1 || { tail -20 $O/tree_small.jsonl; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/r06d/tree_small.jsonl"):
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    keys = [k for k in d if isinstance(d[k], dict)]
    best = sorted(keys, key=lambda k: d[k]["us"])[:3]
    sel = {k: d[k]["us"] for k in keys if k.startswith("split") or k in ("whole_tpt1", "whole_la21_tpt1")}
    print(d["rows"], {k: d[k]["us"] for k in best}, sel)
PY
