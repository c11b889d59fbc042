#!/usr/bin/env bash
# A/B of the batcher idle spin on the REST headline: interleaved runs
OUT=gpurun_out/ab
mkdir -p $OUT
for r in 1 2; do
  for v in 0 50; do
    SCA_IDLE_SPIN_US=$v timeout -k 10 200 python bench.py --steps 20 > $OUT/spin${v}_r$r.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/spin${v}_r$r.log') if l.startswith('{')][-1]); print('spin=$v r=$r', d['value'], d['p50_ms'], d['p99_ms'])"
  done
done
