#!/usr/bin/env bash
# Headline (REST iris): load-generator threads 5 vs 4 alternated, 3 reps, server threads 10.
set -o pipefail
OUT=gpurun_out/thread_ab
mkdir -p $OUT
for rep in 1 2 3; do
  for c in 5 4; do
    timeout -k 10 200 python bench.py --extras none --server-threads 10 --client-threads $c > $OUT/c${c}_r$rep.log 2>&1 || exit $?
    echo "client=$c rep=$rep $(grep -o '"value": [0-9.]*\|"p50_ms": [0-9.]*\|"p99_ms": [0-9.]*\|"server_cpus": [0-9.]*\|"loadgen_cpus": [0-9.]*' $OUT/c${c}_r$rep.log | head -5 | tr '\n' ' ')" | tee -a $OUT/summary.txt
  done
done
timeout -k 10 200 python bench.py --api grpc --extras none --server-threads 10 --client-threads 4 > $OUT/grpc_c4.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --api grpc --extras none --server-threads 10 --client-threads 5 > $OUT/grpc_c5.log 2>&1 || exit $?
for c in 4 5; do echo "grpc client=$c $(grep -o '"value": [0-9.]*\|"p99_ms": [0-9.]*' $OUT/grpc_c$c.log | head -2 | tr '\n' ' ')" | tee -a $OUT/summary.txt; done
