#!/usr/bin/env bash
# PMC passes over the small-batch tree kernels (xgb1000 shape: 1000 trees,
# depth 8, 32 features, 9 rows): the whole-ensemble kernel and the fused
# partial kernel, via tools/tree_microbench.py --small.  One rocprofv3 run per
# counter group within the per-block limits, each under its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/tree_pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
ROWS="${ROWS:-9}"
MB=(python3 "$ROOT/tools/tree_microbench.py" --small --rows "$ROWS" --iters 100)
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- "${MB[@]}" > "$OUT/trace.log" 2>&1 || exit $?
pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc pass $name: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- "${MB[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== pmc pass $name rc=$rc"
  [ $rc -eq 0 ] || { tail -n 20 "$OUT/$name.log"; exit $rc; }
}
pass sq_time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
pass l2_fetch FETCH_SIZE TCC_HIT_sum
pass l2_miss TCC_MISS_sum TCC_REQ_sum
echo "pmc done"
