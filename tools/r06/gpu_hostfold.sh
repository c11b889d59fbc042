# Host-fold split kernel (part sums to the host, no atomics / counter) vs the
# atomic fold, by batch size.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06i}
mkdir -p $O
timeout -k 10 300 python3 tools/tree_microbench.py --small --rows 4,8,16,32,48,64,96 --iters 300 > $O/tree_small.jsonl 2>&1 || { tail -20 $O/tree_small.jsonl; exit 1; }
python3 - <<'PY'
import json
for ln in open("gpurun_out/r06i/tree_small.jsonl"):
    if not ln.startswith("{"): continue
    d = json.loads(ln)
    sel = {k: d[k]["us"] for k in d if isinstance(d[k], dict) and (k.startswith("split8") or k.startswith("split16") or k == "whole_la21_tpt1")}
    errs = {k: d[k].get("max_err") for k in d if isinstance(d[k], dict) and "hostfold" in k}
    print(d["rows"], sel, errs)
PY
