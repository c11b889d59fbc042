# Headline: GPU batches in flight per unit (--slots) at the 10 x 5 thread split.
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
for sl in 4 2 3 6 8 4 2 3 6 8; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none --slots $sl > $O/bench_s$sl.log 2>&1 || exit 1
  python - $O/bench_s$sl.log $sl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); c = d["config"]; pr = c["per_rank"][0]
        print("slots", sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], "rows/b", c["mean_rows_per_gpu_batch"], d["self_check"]["ok"])
PY
done
