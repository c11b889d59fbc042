#!/usr/bin/env bash
# Front-end / batcher parameter sweep for the headline REST bench (1 GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out/sweep
OUT=gpurun_out/sweep/results.jsonl
: > "$OUT"
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -c processor /proc/cpuinfo; } > gpurun_out/sweep/cpu.txt 2>&1
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 240 python bench.py --steps 6 --warmup 1 "$@" > gpurun_out/sweep/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/sweep/$tag.log; [ $rc -ge 124 ] && exit $rc; return; fi
  python - "$tag" >> "$OUT" <<PY
import json,sys
d=json.loads(open("gpurun_out/sweep/$tag.log").read().strip().splitlines()[-1])
c=d["config"]
print(json.dumps({"tag":sys.argv[1],"rps":d["value"],"p50":d["p50_ms"],"p99":d["p99_ms"],"rows":c["mean_rows_per_gpu_batch"],"busy":c["gpu_busy_frac_per_slot"],"cpus":c["host_cpus"]}))
PY
  tail -1 "$OUT"
}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/sweep/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/sweep/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for cfg in ${CONFIGS:-"base::" "base2::" "srv8::--server-threads 8" "srv10::--server-threads 10 --client-threads 5" "slots2::--slots 2" "slots8::--slots 8" "grpc::--api grpc"}; do
  tag=${cfg%%::*}; args=${cfg#*::}; args=${args//_/ }  # "_" separates arguments inside one config word
  run "$tag" $args
done
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sweep/prof -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --step-requests 20000 > gpurun_out/sweep/prof.log 2>&1
  echo "prof rc=$?"
fi
echo done
