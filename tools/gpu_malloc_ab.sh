# Headline A/B: glibc malloc tunables (bigger per-thread caches, no trimming)
# vs the defaults.
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
T='glibc.malloc.tcache_count=2048:glibc.malloc.trim_threshold=268435456:glibc.malloc.mmap_threshold=268435456'
for run in base.1 tun.1 base.2 tun.2 base.3 tun.3; do
  if [ "${run%.*}" = tun ]; then export GLIBC_TUNABLES=$T; else unset GLIBC_TUNABLES; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none > $O/bench_$run.log 2>&1 || exit 1
  python - $O/bench_$run.log $run <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
done
