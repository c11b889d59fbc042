# Spin knobs re-checked at the 10 x 5 split: front-end epoll polling
# (SCA_HTTP_SPIN_US), load-generator polling (SCA_LOADGEN_SPIN_US), pump idle
# spin (SCA_IDLE_SPIN_US).
set -o pipefail
O=gpurun_out/r05sp
mkdir -p $O
run() {
  name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none > $O/bench_$name.log 2>&1 || exit 1
  python - $O/bench_$name.log $name <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{"metric"'):
        d = json.loads(l); pr = d["config"]["per_rank"][0]
        print(sys.argv[2], d["value"], d["p50_ms"], d["p99_ms"], "srv", pr["server_cpus"], "lg", pr["loadgen_cpus"], d["self_check"]["ok"])
PY
}
for i in 1 2; do
  run base.$i X=1
  run http20.$i SCA_HTTP_SPIN_US=20
  run lg50.$i SCA_LOADGEN_SPIN_US=50
  run idle0.$i SCA_IDLE_SPIN_US=0
  run idle200.$i SCA_IDLE_SPIN_US=200
done
