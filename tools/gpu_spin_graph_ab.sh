#!/usr/bin/env bash
# Batcher spin knobs A/B across graph shapes (single model, A/B router over 2
# units, MAB over replicas), interleaved, headline harness.  KNOB is the
# environment variable (default SCA_MAX_SPINNERS), VALUES its settings.
set -o pipefail
OUT=gpurun_out/spin_graph_ab
mkdir -p $OUT
KNOB=${KNOB:-SCA_MAX_SPINNERS}
for r in 1 2; do
  for g in ${GRAPHS:-single abtest mab}; do
    for v in ${VALUES:-2 64}; do
      env $KNOB=$v timeout -k 10 200 python bench.py --graph $g --extras none > $OUT/${g}_${v}_r$r.log 2>&1 || exit $?
      python3 -c "
import json
d=json.loads([l for l in open('$OUT/${g}_${v}_r$r.log') if l.startswith('{')][-1]); r=d['config']['per_rank'][0]
print('$g $KNOB=$v r=$r', round(d['value']), d['p50_ms'], d['p99_ms'], 'server_cpus', r['server_cpus'])"
    done
  done
done
