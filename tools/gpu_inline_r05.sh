# Kernel time of xgb1000 / iris with batch rows in pinned host memory vs HBM
# through the BAR (rocprofv3 stats only: the per-dispatch trace is deleted,
# it would exceed gpurun's copy-back limit), then an A/B of responses posted
# from the pump thread (SCA_INLINE_HANDOFF=1) vs the hand-off thread.
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/micro/xcd_l2_probe 50 > $O/xcd_l2_probe.txt 2>&1 || { cat $O/xcd_l2_probe.txt; exit 1; }
cat $O/xcd_l2_probe.txt
for m in xgb1000 iris; do
  for mode in host bar; do
    (cd /tmp && SCA_BATCH_INPUT=$mode SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_${m}_$mode" -o run --output-format csv -- python "$R/bench.py" --model $m --steps 10 --warmup 3 --extras none > "$R/$O/prof_${m}_$mode.log" 2>&1) || exit 1
    find "$R/$O/prof_${m}_$mode" -name '*kernel_trace.csv' -delete
    find "$R/$O/prof_${m}_$mode" -name '*kernel_stats.csv' -exec head -3 {} \;
  done
done
for m in iris xgb1000; do
  for run in inline.1 base.1 inline.2 base.2 inline.3 base.3; do
    inl=0; [ "${run%.*}" = inline ] && inl=1
    SCA_INLINE_HANDOFF=$inl timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 --extras none > $O/bench_${m}_$run.log 2>&1 || exit 1
    echo "$m $run $(grep '^{' $O/bench_${m}_$run.log | tail -1 | cut -c1-300)"
  done
done
