# Headline front-end / load-generator thread split on the final tree (the
# split was last tuned in round 2, before pump-posted responses).
set -o pipefail
O=gpurun_out/r05x3
mkdir -p $O
for sc in 10x5 10x6 11x5 11x6 12x5 9x6 10x5 10x6 11x5 11x6 12x5 9x6; do
  s=${sc%x*}; c=${sc#*x}
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none --server-threads $s --client-threads $c > $O/bench_$sc.log 2>&1 || exit 1
  python - $O/bench_$sc.log $sc <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
done
