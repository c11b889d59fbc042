#!/usr/bin/env bash
# Headline (REST iris) over server / load-generator thread splits of the rank's 16 CPUs, twice each.
set -o pipefail
OUT=gpurun_out/thread_sweep
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "10 5" "11 4" "12 4" "9 6" "10 4"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --extras none --server-threads $1 --client-threads $2 > $OUT/s$1_c$2_r$rep.log 2>&1 || exit $?
    echo "server=$1 client=$2 rep=$rep $(grep -o '"value": [0-9.]*\|"p99_ms": [0-9.]*\|"server_cpus": [0-9.]*\|"loadgen_cpus": [0-9.]*' $OUT/s$1_c$2_r$rep.log | head -4 | tr '\n' ' ')" | tee -a $OUT/summary.txt
  done
done
