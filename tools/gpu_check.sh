#!/usr/bin/env bash
# One-shot GPU validation run (used through gpurun): gpu tests, smoke, benches,
# rocprofv3 kernel trace.  Each GPU step has its own time limit; test failures
# (rc 1) do not stop later steps, but a crash / abort / timeout does.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
STEPS="${STEPS:-tests smoke bench bench_xgb prof}"

run() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/summary.log"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/summary.log"
  tail -n 5 "$OUT/$name.log" | tee -a "$OUT/summary.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a "$OUT/summary.log"
    exit $rc
  fi
  return 0
}

rocm-smi --showproductname > "$OUT/rocm_smi.log" 2>&1 || true
# rocprofv3 traces stay on the box (a full kernel trace is far beyond what
# gpurun copies back); only the *_stats.csv summaries land in $OUT/<step>/
keep_stats() {
  local name=$1
  mkdir -p "$OUT/$name"
  find "/tmp/prof_trace/$name" -name '*stats*.csv' -exec cp {} "$OUT/$name/" \; 2>/dev/null
  rm -rf "/tmp/prof_trace/$name"
}

for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 180 python __graft_entry__.py smoke ;;
    bench) run bench 400 python bench.py --extra-grpc ;;
    bench_grpc) run bench_grpc 400 python bench.py --api grpc ;;
    bench_xgb) run bench_xgb 400 python bench.py --model xgb1000 ;;  # calibrated step size (>= 4 s window)
    bench_abtest) run bench_abtest 300 python bench.py --graph abtest --steps 5 ;;
    bench_pipeline) run bench_pipeline 300 python bench.py --graph pipeline --steps 5 ;;
    bench_mab) run bench_mab 300 python bench.py --graph mab --steps 5 ;;
    bench_replicas) run bench_replicas 300 python bench.py --graph replicas --steps 5 ;;
    prof)
      export TMPDIR=/tmp
      export SCA_BENCH_CLEAN_EXIT=1  # bench.py ends with os._exit otherwise: rocprofv3 would write nothing
      run prof 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace/prof -o run --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --step-requests 20000
      keep_stats prof ;;
    prof_xgb)
      export TMPDIR=/tmp
      export SCA_BENCH_CLEAN_EXIT=1
      run prof_xgb 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace/prof_xgb -o run --output-format csv -- \
        python3 bench.py --model xgb1000 --steps 3 --warmup 1 --step-requests 10000
      keep_stats prof_xgb ;;
    lstm) run lstm 300 python tools/kernel_microbench.py --only lstm --iters 20 ;;
    tree_small) run tree_small 300 python tools/kernel_microbench.py --only tree_small --iters 200 ;;
    prof_abtest)
      export TMPDIR=/tmp
      export SCA_BENCH_CLEAN_EXIT=1
      run prof_abtest 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace/prof_abtest -o run --output-format csv -- \
        python3 bench.py --graph abtest --steps 3 --warmup 1 --step-requests 20000
      keep_stats prof_abtest ;;
    prof_lstm)
      export TMPDIR=/tmp
      run prof_lstm 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace/prof_lstm -o run --output-format csv -- \
        python3 tools/kernel_microbench.py --only lstm --iters 10
      keep_stats prof_lstm ;;
    maha) run maha 300 python tools/maha_bench.py --p 9 20 32 64 --requests 2000 --threads 16 --out "$OUT/maha.json" ;;
    maha_phase) run maha_phase 300 python -u tools/maha_bench.py --p 9 32 64 --requests 1000 --threads 16 --out "$OUT/maha_phase.json" ;;
    jprobe)  # build first on the CPU: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels tools/micro/jacobi_probe.hip -o tools/micro/jacobi_probe
      run jprobe 120 bash -c 'for p in 9 20 32 64; do ./tools/micro/jacobi_probe $p || exit 1; done' ;;
    xgb_tpt) run xgb_tpt 700 bash tools/gpu_xgb_tpt.sh ;;
    threads) run threads 900 bash tools/gpu_threads_sweep.sh ;;
    maha_jac) SCA_MAHA_RANK1_MAX_P=0 run maha_jac 300 python tools/maha_bench.py --p 9 20 32 --requests 2000 --threads 16 --out "$OUT/maha_jacobi.json" ;;
    maha_hh) SCA_MAHA_RANK1_MAX_P=0 SCA_MAHA_JACOBI_MAX_P=0 run maha_hh 300 python tools/maha_bench.py --p 9 32 64 --requests 2000 --threads 16 --out "$OUT/maha_householder.json" ;;
    prof_maha)
      export TMPDIR=/tmp
      run prof_maha 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace/prof_maha -o run --output-format csv -- \
        python3 tools/maha_bench.py --p 9 64 --requests 1000 --threads 16
      keep_stats prof_maha ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "all done" | tee -a "$OUT/summary.log"
