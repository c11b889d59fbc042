# Round-6: remaining new GPU tests, then xgb1000 serving A/B of the split
# kernel's batch cap (SCA_TREE_SPLIT_ROWS 32 default vs 256) with kernel stats.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06c}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_device_graph.py tests/test_mesh_gpu.py \
  "tests/test_outliers.py::test_mahalanobis_device_concurrent_callers_share_launches" > $O/pytest_new.log 2>&1 || { tail -60 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for SR in 32 256; do
  SCA_TREE_SPLIT_ROWS=$SR timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_xgb_$SR -o run -- python3 bench.py --model xgb1000 --steps 10 --warmup 3 --extras none > $O/xgb_$SR.log 2>&1 || { tail -30 $O/xgb_$SR.log; exit 1; }
  grep '^{' $O/xgb_$SR.log | tail -1 | cut -c1-300
  python3 tools/rocpd_stats.py $O/prof_xgb_$SR/run_results.db --csv $O/xgb_${SR}_stats.csv > /dev/null && head -4 $O/xgb_${SR}_stats.csv
  rm -f $O/prof_xgb_$SR/run_results.db
done
