#!/usr/bin/env bash
# REST front-end A/B: dense-ndarray fast JSON path on/off (SCA_REST_FAST_JSON),
# alternated, headline iris bench each time.
set -o pipefail
OUT=gpurun_out/fastjson_ab
mkdir -p $OUT
for i in 1 2; do
  for f in 1 0; do
    SCA_REST_FAST_JSON=$f timeout -k 10 200 python bench.py --extras none > $OUT/bench_f${f}_$i.log 2>&1 || exit $?
    python3 -c "
import json,sys
l=[x for x in open('$OUT/bench_f${f}_$i.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['config']['per_rank'][0]
print('fast=$f rep=$i', round(d['value']), d['p50_ms'], d['p99_ms'], 'server_cpus', r['server_cpus'], 'us/req', round(r['server_cpus']/d['value']*1e6,2))"
  done
done
