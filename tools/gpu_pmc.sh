#!/usr/bin/env bash
# PMC counter passes over the hot serving kernels (run through gpurun).
# One rocprofv3 run per counter group, each within the per-block limits
# (<= 8 SQ, <= 4 TCC incl. FETCH_SIZE's 3 / WRITE_SIZE's 2, <= 2 GRBM) and its
# own hard time limit; a kernel-trace --stats run gives the durations.  Stops
# at the first failing pass.  Summaries: tools/pmc_summary.py.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
export SCA_PMC=1
ONLY="${ONLY:-tree,vae,mlp,linear}"
ITERS="${ITERS:-20}"

timeout -k 10 240 python3 tools/kernel_microbench.py --only "$ONLY" --iters 50 > "$OUT/microbench.jsonl" 2> "$OUT/microbench.err" || exit $?
cat "$OUT/microbench.jsonl"

timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 tools/kernel_microbench.py --only "$ONLY" --iters "$ITERS" > "$OUT/trace.log" 2>&1 || exit $?

pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc pass $name: $*"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 tools/kernel_microbench.py --only "$ONLY" --iters "$ITERS" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== pmc pass $name rc=$rc"
  [ $rc -eq 0 ] || { tail -n 20 "$OUT/$name.log"; exit $rc; }
}
pass sq_time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
pass sq_lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F32
pass l2_fetch FETCH_SIZE TCC_HIT_sum
pass l2_write WRITE_SIZE TCC_MISS_sum
echo "pmc done"
