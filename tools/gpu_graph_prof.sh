#!/usr/bin/env bash
# Graph variants on 1 GPU (headline harness, --graph abtest / mab / pipeline)
# with the serving process's CPU profile (call paths), to see where the
# router / fan-out paths spend their per-request CPU.
set -o pipefail
OUT=gpurun_out/graph_prof
mkdir -p $OUT
for g in ${GRAPHS:-abtest mab pipeline}; do
  timeout -k 10 200 python bench.py --graph $g --extras none $BENCH_ARGS --cpu-profile $OUT/cpuprof_$g.json --cpu-profile-depth 6 > $OUT/bench_$g.log 2>&1 || exit $?
  python3 -c "
import json
l=[x for x in open('$OUT/bench_$g.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['config']['per_rank'][0]
print('$g', round(d['value']), d['p50_ms'], d['p99_ms'], 'server_cpus', r['server_cpus'], 'us/req', round(r['server_cpus']/d['value']*1e6,2))
p=json.load(open('$OUT/cpuprof_$g.json'))
for f in p['functions'][:25]: print('  %5.1f%%' % (100*f['frac']), f['function'][:110])"
done
