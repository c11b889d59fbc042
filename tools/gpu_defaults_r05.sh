# Final defaults: three plain `python bench.py` runs (the driver's N = 1 call)
# and the xgb1000 serving kernel's per-dispatch percentiles.
set -o pipefail
O=gpurun_out/r05df
mkdir -p $O
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_default_$i.log 2>&1 || exit 1
  grep '^{' $O/bench_default_$i.log | tail -1 | cut -c1-260
done
(cd /tmp && SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/$O/db_xgb" -o run -- python "$R/bench.py" --model xgb1000 --steps 10 --warmup 3 --extras none > "$R/$O/prof_xgb.log" 2>&1) || exit 1
db=$(find "$R/$O/db_xgb" -name '*.db' | head -1)
python tools/rocpd_stats.py "$db" --csv $O/kstats_xgb_default.csv | head -3
rm -rf "$R/$O/db_xgb"
grep '^{' $O/prof_xgb.log | tail -1 | cut -c1-260
