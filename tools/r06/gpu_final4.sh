# Final check on the final tree: full GPU suite, smoke(), headline bench.
set -o pipefail
O=gpurun_out/${R06_OUT:-r06z}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400
