#!/usr/bin/env bash
# Multi-unit graph tail sweep (1 GPU): one bench.py run per configuration,
# one summary line each (value, p50, p99, server/loadgen CPUs).  Config file
# lines: <label> <VAR=value[,...] or X=1> [bench.py args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/ab_sweep"
mkdir -p "$OUT"
GRAPHS="${GRAPHS:-abtest}"
i=0
while read -r label envs args; do
  [ -z "$label" ] && continue
  for g in $GRAPHS; do
    i=$((i+1))
    env $envs timeout -k 10 120 python bench.py --graph "$g" --steps 3 --warmup 1 --extras none $args > "$OUT/$g.$label.log" 2>&1
    rc=$?
    python - "$OUT/$g.$label.log" "$g" "$label" "$rc" <<'PY'
import json, sys
path, g, label, rc = sys.argv[1:]
line = None
for ln in open(path):
    if ln.startswith("{"):
        line = json.loads(ln)
if line is None:
    print(f"{g:8s} {label:24s} rc={rc} no line"); sys.exit(0)
pr = line["config"]["per_rank"][0]
print(f"{g:8s} {label:24s} value={line['value']/1e6:.3f}M p50={line['p50_ms']:.3f} p99={line['p99_ms']:.3f} "
      f"srv_cpu={pr['server_cpus']} lg_cpu={pr['loadgen_cpus']} rows/batch={line['config']['mean_rows_per_gpu_batch']}")
PY
    [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  done
done < "${1:-tools/ab_sweep.conf}"
