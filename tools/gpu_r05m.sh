# Full GPU suite with responses posted from the pump (now the default), then
# batch rows in HBM through the BAR vs pinned host rows (SCA_BATCH_INPUT) on
# top of it, and per-dispatch kernel-time percentiles (rocpd database,
# summarised on the box, then deleted: too large to copy back).
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for m in xgb1000 iris; do
  for run in host.1 bar.1 host.2 bar.2 host.3 bar.3; do
    mode=${run%.*}
    SCA_BATCH_INPUT=$mode timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 --extras none > $O/bench_${m}_$run.log 2>&1 || exit 1
    echo "$m $run $(grep '^{' $O/bench_${m}_$run.log | tail -1 | cut -c1-200)"
  done
done
for m in xgb1000 iris; do
  for mode in host bar; do
    (cd /tmp && SCA_BATCH_INPUT=$mode SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/$O/db_${m}_$mode" -o run -- python "$R/bench.py" --model $m --steps 10 --warmup 3 --extras none > "$R/$O/prof_${m}_$mode.log" 2>&1) || exit 1
    db=$(find "$R/$O/db_${m}_$mode" -name '*.db' | head -1)
    python tools/rocpd_stats.py "$db" --csv $O/kstats_${m}_$mode.csv | head -3
    rm -rf "$R/$O/db_${m}_$mode"
  done
done
