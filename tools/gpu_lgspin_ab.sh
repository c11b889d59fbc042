# Headline: load generator polling 50 us before blocking (SCA_LOADGEN_SPIN_US=50) vs blocking, 4 rounds.
set -o pipefail
O=gpurun_out/r05lg
mkdir -p $O
for i in 1 2 3 4; do
  for mode in base lg50; do
    if [ $mode = lg50 ]; then export SCA_LOADGEN_SPIN_US=50; else unset SCA_LOADGEN_SPIN_US; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none > $O/bench_$mode.$i.log 2>&1 || exit 1
    python - $O/bench_$mode.$i.log $mode.$i <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
  done
done
