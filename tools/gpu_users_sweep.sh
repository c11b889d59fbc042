#!/usr/bin/env bash
# Throughput / latency vs closed-loop concurrency (headline graph, 1 GPU):
# one bench line per (api, users) under gpurun_out/users/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/users"
mkdir -p "$OUT"
for api in rest grpc; do
  for u in 16 64 256 1024; do
    timeout -k 10 200 python bench.py --extras none --api $api --users $u --steps 6 --warmup 1 > "$OUT/${api}_$u.log" 2>&1 || exit $?
    echo "$api users=$u $(tail -n 1 "$OUT/${api}_$u.log" | cut -c1-160)"
  done
done
