# Headline placement A/B: load generator on its own cores (SCA_BENCH_LG_CORES=k,
# both SMT threads) vs sharing the rank's CCD with the server threads.
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
for run in 0.1 2.1 3.1 0.2 2.2 3.2; do
  SCA_BENCH_LG_CORES=${run%.*} timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none > $O/bench_lg$run.log 2>&1 || exit 1
  python - $O/bench_lg$run.log $run <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print("lg_cores", sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
done
