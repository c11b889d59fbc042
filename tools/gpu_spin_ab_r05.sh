# A/B: epoll spin before blocking in the HTTP front end (SCA_HTTP_SPIN_US)
# and in the load generator (SCA_LOADGEN_SPIN_US).  Headline bench, 2 runs each.
set -o pipefail
mkdir -p gpurun_out/r05g
run() {  # tag, env...
  local tag=$1; shift
  for i in 1 2; do
    env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras none > gpurun_out/r05g/$tag.$i.log 2>&1 || return 1
    python - "$tag" "$i" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/r05g/{sys.argv[1]}.{sys.argv[2]}.log") if x.startswith('{')][-1]
d=json.loads(l); r=d['config']['per_rank'][0]
print(sys.argv[1], sys.argv[2], round(d['value']), d['p50_ms'], d['p99_ms'], 'server_cpus', r['server_cpus'], 'loadgen_cpus', r['loadgen_cpus'], flush=True)
PY
  done
}
run base X=0 && run lg50 SCA_LOADGEN_SPIN_US=50 && run srv20 SCA_HTTP_SPIN_US=20 && run both SCA_LOADGEN_SPIN_US=50 SCA_HTTP_SPIN_US=20 && run lg1000 SCA_LOADGEN_SPIN_US=1000
