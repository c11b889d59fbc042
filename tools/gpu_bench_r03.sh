#!/usr/bin/env bash
# r03 GPU check of the reworked bench: the driver's exact 1-GPU command, then
# every in-process variant child folded onto the one GPU (code-path rehearsal
# of the multi-GPU graphs; per-GPU numbers need the 8-GPU node).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out/r03b"
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_n1.log" 2>&1
rc=$?; echo "bench_n1 rc=$rc"; tail -c 3000 "$OUT/bench_n1.log"
[ $rc -eq 0 ] || exit $rc
for v in abtest pipeline mab replicas; do
  span=2; [ $v = pipeline ] && span=4; [ $v = mab ] && span=4; [ $v = replicas ] && span=4
  DL=$(python3 -c "import time; print(time.time()+90)")
  SCA_BENCH_FOLD=1 timeout -k 10 100 python3 bench.py --variant-child $v --span $span --deadline $DL > "$OUT/variant_$v.log" 2>&1
  rc=$?; echo "variant $v rc=$rc"; tail -c 1500 "$OUT/variant_$v.log"; echo
  [ $rc -eq 0 ] || exit $rc
done
echo done
