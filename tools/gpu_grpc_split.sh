# gRPC headline at the 10 x 4 and 10 x 5 thread splits.
set -o pipefail
O=gpurun_out/r05g2
mkdir -p $O
for sc in 10x4 10x5 10x4 10x5 10x6; do
  s=${sc%x*}; c=${sc#*x}
  timeout -k 10 200 python bench.py --api grpc --steps 20 --warmup 5 --extras none --server-threads $s --client-threads $c > $O/grpc_$sc.log 2>&1 || exit 1
  python - $O/grpc_$sc.log $sc <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["metric"][:40], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
done
