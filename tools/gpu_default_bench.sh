#!/usr/bin/env bash
# The driver's invocation (no flags) and the xgb1000 config, at HEAD.
set -o pipefail
OUT=gpurun_out/default_bench
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --model xgb1000 --step-requests 20000 > $OUT/bench_xgb.log 2>&1 || exit $?
for f in bench bench_xgb; do echo "$f $(grep -o '"value": [0-9.]*\|"p50_ms": [0-9.]*\|"p99_ms": [0-9.]*\|"client_threads": [0-9]*' $OUT/$f.log | tr '\n' ' ')"; done
