set -o pipefail
mkdir -p gpurun_out
for t in 9 10 11 12; do
  timeout -k 10 200 python bench.py --server-threads $t --steps 10 --warmup 2 > gpurun_out/thr_$t.log 2>&1 || exit 1
  python3 -c "
import json
l=[json.loads(x) for x in open('gpurun_out/thr_$t.log') if x.startswith('{')][-1]
print('threads=$t', l['value'], l['p50_ms'], l['p99_ms'], l['config']['per_rank'][0]['server_cpus'], l['config']['per_rank'][0]['loadgen_cpus'])"
done
