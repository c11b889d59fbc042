# Batch rows staged in HBM through the BAR (SCA_BATCH_INPUT=bar) vs pinned
# host memory: the probe, GPU serving tests with bar on, REST A/B for the
# headline (iris) and xgb1000, responses posted from the pump (SCA_INLINE_HANDOFF)
# vs the hand-off thread, and a kernel trace of xgb1000 with bar on.
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mesh_gpu.py tests/test_serve_multi.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_mesh_fine.log 2>&1 || { tail -40 $O/pytest_mesh_fine.log; exit 1; }
tail -2 $O/pytest_mesh_fine.log
timeout -k 10 60 ./tools/micro/vram_probe 4000 9 32 > $O/probe_9x32.txt 2>&1 || { cat $O/probe_9x32.txt; exit 1; }
cat $O/probe_9x32.txt
timeout -k 10 60 ./tools/micro/vram_probe 4000 64 32 > $O/probe_64x32.txt 2>&1 || exit 1
grep -q '"fine_grained_cpu_writable": true' $O/probe_9x32.txt || { echo "BAR not CPU-writable: stop"; exit 0; }
grep -q '"src": "vram".*"mismatches": 0' $O/probe_9x32.txt || { echo "BAR path mismatches: stop"; exit 0; }
SCA_BATCH_INPUT=bar timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_serving.py tests/test_batcher_signal_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_bar.log 2>&1 || { tail -30 $O/pytest_bar.log; exit 1; }
tail -2 $O/pytest_bar.log
for m in iris xgb1000; do
  for run in host.1 bar.1 host.2 bar.2; do
    mode=${run%.*}
    SCA_BATCH_INPUT=$mode timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 --extras none > $O/bench_${m}_$run.log 2>&1 || exit 1
    echo "$m $run $(grep '^{' $O/bench_${m}_$run.log | tail -1 | cut -c1-330)"
  done
done
for run in inline.1 base.1 inline.2 base.2; do
  inl=0; [ "${run%.*}" = inline ] && inl=1
  SCA_INLINE_HANDOFF=$inl timeout -k 10 200 python bench.py --model iris --steps 20 --warmup 5 --extras none > $O/bench_iris_$run.log 2>&1 || exit 1
  echo "iris $run $(grep '^{' $O/bench_iris_$run.log | tail -1 | cut -c1-330)"
done
cd /tmp && SCA_BATCH_INPUT=bar SCA_BENCH_CLEAN_EXIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o xgb_bar --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --model xgb1000 --steps 10 --warmup 3 --extras none > "$GRAFT_REPO_ROOT/$O/prof_xgb.log" 2>&1
