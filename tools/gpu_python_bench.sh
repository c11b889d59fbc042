#!/usr/bin/env bash
# Python-runtime benches on the GPU box's 16-CPU share (user Python classes,
# the reference's wrapper-microservice workload): one line per mode.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/pybench"
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 180 python bench.py --extras none --steps 5 --warmup 1 --step-requests 20000 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(tail -n 1 "$OUT/$name.log" | cut -c1-400)"
  [ $rc -eq 0 ] || exit $rc
}
run noop_inproc --model python-noop --py-batching 0
run noop_batched --model python-noop
run iris_inproc --model python-iris --py-batching 0
run iris_batched --model python-iris
run iris_pool8 --model python-iris --py-batching 0 --py-workers 8
run iris_pool4_batched --model python-iris --py-workers 4
