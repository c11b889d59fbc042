# Round-6: the new GPU paths (MFMA linear, one-kernel linear graphs, mesh peer
# probe + fallback, Mahalanobis step order) + linear kernel A/B under rocprof.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06b}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "linear" tests/test_device_graph.py tests/test_mesh_gpu.py \
  "tests/test_outliers.py::test_mahalanobis_device_concurrent_callers_share_launches" -m gpu > $O/pytest_new.log 2>&1 || { tail -60 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_linear -o run -- python3 tools/r06/linear_bench.py > $O/linear_bench.log 2>&1 || { tail -30 $O/linear_bench.log; exit 1; }
cat $O/linear_bench.log | grep '^{'
